"""Worker spawning and the per-rank training loop.

Reference: the parent clones/chunks parameters onto every GPU, spawns one ``multiprocessing.Process`` per
GPU (spawn start method) whose children receive CUDA tensors through IPC handles, joins them **without
checking exit codes**, and reads the children's in-place updates back (train_ffns.py:174-193, 262-287,
315-338).

Here the parent ships only the (small) config; every rank builds its own shard of the parameters
deterministically (same CPU generator stream as the reference, or the device Philox stream), trains,
and rank 0 returns a result record (timings, parameter slices, optionally the full gathered parameters)
through a queue.  Exit codes are checked: a failed rank terminates the others and raises in the parent,
and every collective has a timeout.  ``run_rank`` is also the body used under ``torchrun`` (bench.py).
"""
from __future__ import annotations

import dataclasses
import os
import time
import traceback

import torch
import torch.multiprocessing as mp

from ..utils.config import METHODS, ModelConfig, TrainConfig
from ..utils.data import make_data, stripe_seeds
from ..utils.metrics import StepTimer, flops_per_step

METHOD_MESH = {  # method -> (dp_mode, dp, tp) given n ranks
    1: lambda n, a: ("none", 1, 1),
    2: lambda n, a: ("ddp", n, 1),
    3: lambda n, a: ("fsdp", n, 1),
    4: lambda n, a: ("none", 1, n),
    5: lambda n, a: (a.get("hybrid_dp_mode", "fsdp"), n // a["tp"], a["tp"]),
    6: lambda n, a: ("zero", n, 1),
}


def method_ranks(method: int, n: int) -> int:
    return 1 if method == 1 else n


def build_params(cfg: TrainConfig, init: str, seed: int, device) -> list[dict]:
    from ..models.ffn import init_ffn_layer, init_ffn_params_device

    m = cfg.model
    if init == "cpu_compat":
        gen = torch.Generator()
        gen.manual_seed(seed)
        torch.randint(100_000, (cfg.num_steps,), generator=gen)  # the reference draws seeds first (:360)
        return [init_ffn_layer(m.D, m.F, gen, m.gated) for _ in range(m.layers)]
    return init_ffn_params_device(m.D, m.F, m.layers, seed, device, m.gated)


def draw_seeds(cfg: TrainConfig, seed: int) -> torch.Tensor:
    gen = torch.Generator()
    gen.manual_seed(seed)
    return torch.randint(100_000, (cfg.num_steps,), generator=gen)


def run_rank(rank: int, world: int, cfg_dict: dict, method: int, backend: str, port: int, opts: dict,
             queue=None) -> dict | None:
    """Body of one rank: init comm, build mesh + engine, train, report.  Returns rank 0's record."""
    from ..utils.checkpoint import load_into, save_checkpoint
    from ..utils.profiling import maybe_profile
    from .engine import FFNTrainer
    from .mesh import Mesh, init_distributed

    cfg = _cfg_from_dict(cfg_dict)
    # opts["device"] == "cuda" with gloo: several ranks share one GPU (RCCL refuses two ranks on one device), so
    # the multi-rank engine paths run with the HIP kernels and streams, collectives staged through the host
    use_gpu = backend == "nccl" or opts.get("device") == "cuda"
    if use_gpu:
        # keep every later stream (torch's pool: engine side streams, process-group streams) off the compute stream's
        # hardware queue, on every GPU path incl. world == 1 and gloo-on-cuda ranks (init_distributed does it for
        # nccl); before anything creates streams
        from ..utils.streams import reserve_compute_queue

        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", rank)) % max(1, torch.cuda.device_count()))
        reserve_compute_queue(torch.cuda.current_device())
    if world > 1 or opts.get("force_dist"):
        init_distributed(backend, rank, world, "127.0.0.1", port)
    device = torch.device("cuda", torch.cuda.current_device()) if use_gpu else torch.device("cpu")
    if use_gpu and world == 1:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
        device = torch.device("cuda", torch.cuda.current_device())
    dp_mode, dp, tp = METHOD_MESH[method](world, opts)
    cfg.dp_mode, cfg.dp, cfg.tp = dp_mode, dp, tp
    mesh = Mesh.build(dp, tp, separate_streams=cfg.separate_streams, force=cfg.force_comm,
                      comm_backend=cfg.comm_backend, device=device if device.type == "cuda" else None)
    eng = FFNTrainer(cfg, mesh, device)

    seed = int(opts.get("seed", 0))
    init = opts.get("init", "cpu_compat")
    if opts.get("params") is not None:  # caller-provided logical parameters (api.train_* entry points)
        eng.load_full_params([{k: torch.as_tensor(v) for k, v in p.items()} for p in opts["params"]])
    else:
        eng.load_full_params(build_params(cfg, init, seed, device))
    seeds = torch.as_tensor(opts["seeds"], dtype=torch.int64) if opts.get("seeds") is not None \
        else draw_seeds(cfg, seed)
    my_seeds = stripe_seeds(seeds, dp, mesh.dp_rank) if dp > 1 else seeds
    start_step, ckpt_read = 0, 0
    if opts.get("resume"):
        meta, ckpt_read = load_into(eng, opts["resume"])
        start_step = int(meta["step"])
    data = make_data(cfg.data, cfg.tokens, cfg.model.D, cfg.torch_dtype, device)
    if hasattr(data, "bind_transposed"):
        data.bind_transposed(*eng.input_transposes())
    timer = StepTimer(device)
    stop_after = int(opts.get("stop_after") or len(my_seeds))
    done = start_step
    seed_list = my_seeds.tolist()
    depth = max(1, getattr(data, "depth", 1))  # host threads drawing upcoming batches (cpu_compat data)
    limit = min(len(seed_list), stop_after)
    for k in range(start_step, min(start_step + depth, limit)):
        data.prefetch(int(seed_list[k]))
    from contextlib import nullcontext

    from .comm import count_collectives

    counter = count_collectives() if opts.get("count_collectives") else nullcontext()
    try:
        with maybe_profile(opts.get("profile", ""), rank), counter:
            for i, s in enumerate(seed_list):
                if i < start_step:
                    continue
                if i >= stop_after:
                    break
                _maybe_inject_fault(rank, i)
                timer.start()
                nxt = seed_list[i + depth] if i + depth < limit else None
                x, dy = data.fill(int(s), next_seed=nxt)
                eng.train_step(x, dy)
                timer.stop()
                done = i + 1
    except BaseException:
        # error path: abort native communicators (no synchronising teardown against a dead peer) and
        # let the parent see the failure; torch process groups time out / are torn down with the process
        mesh.destroy(abort=True)
        raise
    timer.finish()
    eng.check_health()
    # peak of training itself: read before the checkpoint export / parameter gather, which materialise transient
    # full fp32 copies of split masters that never exist during a step
    peak_hbm = torch.cuda.max_memory_allocated(device) / 2**30 if device.type == "cuda" else 0.0
    if opts.get("ckpt_dir"):
        save_checkpoint(eng, opts["ckpt_dir"], step=done, fmt=opts.get("ckpt_format", "consolidated"),
                        meta={"method": method, "seed": seed, "cfg": cfg_dict})
    full = eng.gather_full_params() if opts.get("return_params", True) else None
    read_max = ckpt_read
    if world > 1 or opts.get("force_dist"):
        import torch.distributed as dist

        t = torch.tensor([ckpt_read], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        read_max = int(t.item())
    rec = None
    if rank == 0:
        steps = done - start_step
        rec = {
            "method": method, "name": METHODS[method], "world": world, "steps": steps,
            "step_ms": timer.step_ms, "steady_ms": timer.steady_ms,
            "tokens_per_step_global": cfg.tokens * dp,
            "flops_per_step_rank": flops_per_step(cfg, tp=tp, recompute=cfg.recompute),
            "shapes": [(tuple(p["w1"].shape), tuple(p["w2"].shape)) for p in full] if full else None,
            "slices": [(p["w1"][:5, :5].clone(), p["w2"][:5, :5].clone()) for p in full] if full else None,
            "params": full if opts.get("return_full", False) else None,
            "peak_hbm_gib": peak_hbm,
            # per-rank persistent state (elements): ZeRO keeps 1/dp of the fp32 master / moments
            "state_numel": {"master": eng.master_numel, "total": eng.total, "copy": eng.copy.numel(),
                            "grads": eng.grads.numel(),
                            "adam": eng.adam_m.numel() if getattr(eng, "adam_m", None) is not None else 0},
            "ckpt_bytes_read_max": read_max,
            # GEMM layouts the engine chose (parallel/engine.py): NN weight gradients, W2 stored transposed
            "layout": {"wgrad_nn": bool(eng.wgrad_nn), "wgrad_nn_w2": bool(eng.wgrad_nn_w2), "w2t": bool(eng.w2t),
                       "tp_transposed": bool(eng.tmode)},
        }
        if opts.get("count_collectives") and steps > 0:
            rec["collectives_per_step"] = {r: c / steps for r, c in counter.by_role(mesh.groups).items()}
    if world > 1 or opts.get("force_dist"):
        import torch.distributed as dist

        dist.barrier()
        mesh.destroy()
        dist.destroy_process_group()
    if queue is not None and rank == 0:
        queue.put(("ok", to_numpy(rec)))  # by-value payload: survives the worker's exit
    return rec


class InjectedFault(RuntimeError):
    pass


def _maybe_inject_fault(rank: int, step: int) -> None:
    """Fault injection: ``DLLM_FAULT_RANK=k DLLM_FAULT_STEP=s`` makes rank k fail at step s
    (``DLLM_FAULT_MODE=exit`` kills the process instead of raising) to test failure propagation."""
    fr, fs = os.environ.get("DLLM_FAULT_RANK"), os.environ.get("DLLM_FAULT_STEP")
    if fr is None or int(fr) != rank or int(fs or 0) != step:
        return
    if os.environ.get("DLLM_FAULT_MODE") == "exit":
        os._exit(17)
    raise InjectedFault(f"injected fault on rank {rank} at step {step}")


def to_numpy(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu().numpy()
    if isinstance(obj, dict):
        return {k: to_numpy(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(to_numpy(v) for v in obj)
    return obj


def to_torch(obj):
    import numpy as np

    if isinstance(obj, np.ndarray):
        return torch.from_numpy(obj)
    if isinstance(obj, dict):
        return {k: to_torch(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(to_torch(v) for v in obj)
    return obj


def _cfg_from_dict(d: dict) -> TrainConfig:
    d = dict(d)
    m = ModelConfig(**d.pop("model"))
    return TrainConfig(model=m, **d)


def cfg_to_dict(cfg: TrainConfig) -> dict:
    return dataclasses.asdict(cfg)


def _entry(rank, world, cfg_dict, method, backend, port, opts, queue):
    try:
        os.environ["LOCAL_RANK"] = str(rank)
        run_rank(rank, world, cfg_dict, method, backend, port, opts, queue)
    except BaseException as e:  # report then exit non-zero
        queue.put(("err", f"rank {rank}: {type(e).__name__}: {e}\n{traceback.format_exc()}"))
        raise


def spawn(nprocs: int, cfg: TrainConfig, method: int, backend: str, port: int, opts: dict,
          timeout_s: float = 3600.0) -> dict:
    """Run ``nprocs`` ranks in spawned processes; returns rank 0's record or raises on any failure."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    cfg_dict = cfg_to_dict(cfg)
    if nprocs == 1 and backend != "gloo":
        # in-process single rank (the reference's train_1gpu also runs in the parent, :101-116)
        return run_rank(0, 1, cfg_dict, method, backend, port, opts)
    procs = [ctx.Process(target=_entry, args=(r, nprocs, cfg_dict, method, backend, port, opts, q))
             for r in range(nprocs)]
    for p in procs:
        p.start()
    result, err = None, None
    deadline = time.time() + timeout_s
    while True:
        try:
            kind, payload = q.get(timeout=0.5)
            if kind == "ok":
                result = payload
            else:
                err = err or payload
        except Exception:
            pass
        codes = [p.exitcode for p in procs]
        if err is not None or any(c not in (None, 0) for c in codes):
            for p in procs:
                if p.is_alive():
                    p.terminate()
            for p in procs:
                p.join(10)
            raise RuntimeError(err or f"worker failed with exit codes {codes}")
        if all(c == 0 for c in codes):
            # drain a result that may have been queued just before exit
            while result is None:
                try:
                    kind, payload = q.get(timeout=2.0)
                except Exception:
                    break
                if kind == "ok":
                    result = payload
            break
        if time.time() > deadline:
            for p in procs:
                p.terminate()
            raise TimeoutError("workers did not finish in time")
    for p in procs:
        p.join()
    return to_torch(result)
