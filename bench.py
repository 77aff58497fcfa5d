"""Flagship benchmark: FFN-stack training throughput (whole-node tokens/s) on MI355X.

Metric/config from BASELINE.json: "FFN tokens/sec (whole node) at hidden=4096 for DDP/FSDP/MP, 1/2/4/8
MI355X" on the 8-layer hidden=4096 FFN stack (FFN = 4·hidden = 16384, ReLU, as train_ffns.py:361),
batch 8 × seq 1024 = 8192 tokens per rank per step, bf16 compute with fp32 master weights, SGD (the
reference optimizer, train_ffns.py:172), random-init weights and synthetic device-generated data.

    python bench.py --gpus N --steps K --warmup W            # N=1 in-process; N>1: starts its own N ranks
    torchrun --nproc-per-node N bench.py --gpus N ...          # one rank per GPU over RCCL/xGMI

With N > 1 and no launcher environment (no ``WORLD_SIZE``), the process launches its own N ranks the way the
reference's ``train_ffns.py`` does (one worker per GPU from a plain ``python`` command, train_ffns.py:184-191,
:375): fresh child interpreters with ``RANK``/``LOCAL_RANK``/``WORLD_SIZE``/``MASTER_*`` set, started before this
process imports torch (so it never touches HIP), rank 0's stdout relayed, any failing rank failing the run.

Each timed step is the full training step: device mock-data generation, forward, backward (all weight
and input gradients except the unused layer-0 input grad), gradient communication and the optimizer
update.  K steps are bracketed by cuda synchronize + barrier on both sides; the max over ranks is
reported; rank 0 prints ONE JSON line.

Headline (``value``): ``--method`` (default ``zero``) on the 8-layer stack.  ``zero`` is data parallel
with DDP semantics (identical updates to DDP: summed gradients, every rank's replica updated) carried
as ZeRO-2: bucketed bf16 gradient reduce-scatter overlapped with the backward, fp32 master / optimizer
state sharded 1/N, bf16 weight all-gather overlapped with the next forward.  With N=1 there is no
gradient collective and the SGD update is fused into the weight-gradient GEMM epilogues (``dp1``).

``methods``: the reference's methods timed side by side like its ``--method 0`` (train_ffns.py:373-384),
each on its own engine at the same N, with steady-state tokens/s, ms/step, peak HBM and (when the method
communicates) per-role collective time and the fraction of it hidden under the GEMMs (comm observer,
utils/observe.py, measured on extra steps after the timed ones):

* ``ddp``   bucketed gradient all-reduce + full optimizer on every rank (train_ffns.py:156-193);
* ``zero``  as the headline;
* ``fsdp``  ZeRO-3 row shards, prefetched all-gathers, async reduce-scatter (train_ffns.py:197-287);
* ``tp``    the MP config of BASELINE.json: hidden 4096, FFN 14336, one layer, column/row split over the
            N GPUs (train_ffns.py:290-338; every rank sees every token: strong scaling);
* ``hybrid`` BASELINE config 5: the Llama-3-8B-dims FFN stack (hidden 4096, FFN 14336, SwiGLU/SiLU, 32 layers)
            on an FSDP x TP mesh (TP = min(N, 2) or ``--tp``; 8192 tokens per FSDP rank).

At N=1 the ddp/zero/fsdp/tp/hybrid entries run their collective code paths over size-1 communicators
(``force_comm``), so each method's own overhead is visible even on one GPU.  Weak scaling for the DP
methods: every rank processes 8192 tokens per step (global batch = 8·N sequences).
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time


def _requested_ranks(argv) -> int:
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument("--gpus", type=int, default=0)
    return p.parse_known_args(argv)[0].gpus


def self_launch(argv, n: int, grace_s: float = 30.0) -> int:
    """Start ``n`` ranks of this script as child interpreters (stdlib only: no torch / HIP in this process) and
    wait for them.  Rank 0 keeps this process's stdout (the one JSON line); the other ranks' stdout goes to stderr.
    The first rank that fails ends the others after ``grace_s`` (they may be blocked in a collective with it);
    the exit code is the first non-zero rank exit code, or 0.  SIGTERM/SIGINT are forwarded to every rank."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DLLM_SELF_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                      stdout=None if r == 0 else sys.stderr))

    def forward(sig, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)

    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    rc, failed_at = 0, None
    while any(p.poll() is None for p in procs):
        for r, p in enumerate(procs):
            if p.returncode not in (None, 0) and rc == 0:
                rc, failed_at = p.returncode, time.monotonic()
                print(f"bench.py: rank {r} exited with {p.returncode}", file=sys.stderr, flush=True)
        if failed_at is not None and time.monotonic() - failed_at > grace_s:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        time.sleep(0.2)
    for r, p in enumerate(procs):
        if p.returncode != 0 and rc == 0:
            rc = p.returncode
            print(f"bench.py: rank {r} exited with {p.returncode}", file=sys.stderr, flush=True)
    return rc if rc >= 0 else 128 - rc  # a rank killed by signal k -> 128 + k


if __name__ == "__main__" and "WORLD_SIZE" not in os.environ and _requested_ranks(sys.argv[1:]) > 1:
    sys.exit(self_launch(sys.argv[1:], _requested_ranks(sys.argv[1:])))

import torch  # noqa: E402

import dllm  # noqa: F401,E402
from dllm.parallel import comm  # noqa: E402
from dllm.parallel.engine import FFNTrainer  # noqa: E402
from dllm.parallel.mesh import Mesh, init_distributed  # noqa: E402
from dllm.utils.config import ModelConfig, TrainConfig  # noqa: E402
from dllm.utils.data import DeviceMockData  # noqa: E402
from dllm.utils.metrics import flops_per_step, peak_tflops  # noqa: E402

METRIC = "FFN tokens/sec (whole node) at hidden=4096 for DDP/FSDP/MP, 1/2/4/8 MI355X"
MP_FFN = 14336  # BASELINE.json config 4: FFN (hidden=4096, ffn=14336) MP column/row split


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=0)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--method", choices=["ddp", "zero", "fsdp", "tp", "hybrid"], default="zero",
                   help="headline method (see module docstring); zero = DDP semantics as ZeRO-2")
    p.add_argument("--methods", default="ddp,zero,fsdp,tp,hybrid",
                   help="comma list of methods also timed side by side ('' or 'none' = headline only)")
    p.add_argument("--method_steps", type=int, default=0,
                   help="minimum timed steps per side-by-side method (0 = min(steps, 10)); see --side_timed_ms")
    p.add_argument("--side_warmup_ms", type=float, default=150.0,
                   help="side-by-side methods: after min(warmup, 3) steps keep warming up until this much step time "
                        "has run (the GPU clock ramps over its first ~50 ms of load, profiles/r4/window_probe_r4.txt)")
    p.add_argument("--side_timed_ms", type=float, default=300.0,
                   help="side-by-side methods: time at least max(method steps, ceil(this / step time)) steps")
    p.add_argument("--side_max_steps", type=int, default=1000,
                   help="cap on the timed steps of one side-by-side method")
    p.add_argument("--side_deadline_s", type=float, default=420.0,
                   help="wall-clock budget of the side-by-side methods after the headline (0 = none): past it, rank 0 "
                        "prints the line with the methods finished so far and every rank exits")
    p.add_argument("--observe_steps", type=int, default=2,
                   help="extra steps per communicating method under the comm observer (0 = off)")
    p.add_argument("--tp", type=int, default=0, help="TP degree for --method hybrid")
    p.add_argument("--model_size", type=int, default=4096)
    p.add_argument("--ffn_dim", type=int, default=0)
    p.add_argument("--mp_ffn_dim", type=int, default=MP_FFN, help="FFN width of the tp (MP) method entry")
    p.add_argument("--mp_layers", type=int, default=1, help="layers of the tp (MP) method entry")
    p.add_argument("--llama_ffn_dim", type=int, default=14336,
                   help="FFN width of the hybrid method entry (BASELINE config 5: Llama-3-8B dims, SwiGLU)")
    p.add_argument("--llama_layers", type=int, default=32, help="layers of the hybrid method entry")
    p.add_argument("--layers", type=int, default=8)
    p.add_argument("--batch_size", type=int, default=8)
    p.add_argument("--seq_len", type=int, default=1024)
    p.add_argument("--act", default="relu")
    p.add_argument("--gated", action="store_true")
    p.add_argument("--dtype", default="bf16")
    p.add_argument("--grad_dtype", default="bf16",
                   help="gradient / gradient-collective dtype for N>1 (N=1 fuses the fp32 update into the GEMM)")
    p.add_argument("--optimizer", default="sgd")
    p.add_argument("--bucket_mb", type=float, default=0.0)
    p.add_argument("--recompute", default="none")
    p.add_argument("--sequence_parallel", action="store_true")
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--init_scale", default="auto",
                   help="weight init std: a number, 'fan_in' (1/sqrt(fan_in) per matrix), or 'auto' = fan_in.  The "
                        "reference's fixed 2e-2 (--init_scale 0.02) grows activations ~2.3x per layer at D=4096: the "
                        "8-layer flagship stack reaches y std ~830 and its first SGD update overflows the weights to "
                        "inf / NaN, after which the GEMMs run on inf / NaN / zero-filled data -- and on MI355X, whose "
                        "clock is power-limited, MFMA throughput depends on the data (28.3 vs 35.0 ms per step).  The "
                        "headline therefore trains on finite data; the reference-init timing is reported next to it "
                        "(reference_init)")
    p.add_argument("--no_reference_init", action="store_true",
                   help="skip the headline's second run with the reference's 2e-2 init (the reference_init field)")
    p.add_argument("--json_out", default="")
    p.add_argument("--comm", choices=["torch", "native"], default="torch",
                   help="role communicators: torch ProcessGroupNCCL or the native C++ RCCL layer")
    p.add_argument("--backend", choices=["nccl", "gloo", "gloo_gpu"], default="nccl",
                   help="gloo = CPU dry run of the multi-rank path (tests; tiny dims); gloo_gpu = the N-rank path "
                        "with the HIP kernels on the GPU(s) and gloo collectives on device tensors, so N ranks may "
                        "share one GPU (RCCL refuses that): a plumbing rehearsal of the N>1 bench, not a measurement")
    p.add_argument("--graph", action="store_true",
                   help="capture the whole step (data + fwd + bwd + fused SGD) in a HIP graph (N=1 path)")
    p.add_argument("--side_opt", type=int, default=0,
                   help="N=1: store wgrads and run SGD on a side stream over this many workgroups (0 = fuse the "
                        "update into the wgrad GEMM epilogue; -1 = each weight's flat update, any optimizer, on the "
                        "side stream with the whole chip)")
    p.add_argument("--phases", action="store_true",
                   help="also report per-phase GPU time (forward / backward / optimizer tail) from HIP events")
    p.add_argument("--wgrad_layout", choices=["auto", "tn", "nn", "nn_w1", "nn_w2t"], default="auto",
                   help="weight-gradient GEMM layout: nn = transposed xᵀ / dyᵀ copies written by the producing "
                        "epilogues, both weight gradients as NN GEMMs with a K-contiguous A (models/ffn.NNWgrad); "
                        "auto = nn wherever the engine supports it")
    p.add_argument("--w2_storage", choices=["auto", "rowmajor", "transposed"], default="auto",
                   help="W2 storage in the row-major layer: auto = W2ᵀ with the NN weight-gradient layout and on TP layers "
                        "(the dgrad then runs NT), rowmajor = [D, F] everywhere")
    p.add_argument("--tp_allreduce", choices=["rccl", "custom", "auto"], default="rccl",
                   help="TP activation all-reduce: RCCL, the custom two-shot xGMI peer all-reduce (csrc/car.hip), or auto "
                        "(both timed on the [T, D] message at engine build on the real tp group, the faster kept; "
                        "the timings go to the method's tp_allreduce_choice)")
    p.add_argument("--gemm_variant", default="auto",
                   choices=["auto", "2stage", "8phase", "8phase_stagger", "4phase_stagger", "pp"],
                   help="bf16 GEMM main-loop schedule (auto = 8-phase staggered when K %% 128 == 0; pp = 256x128 tiles, "
                        "two blocks per CU)")
    p.add_argument("--tpb", type=int, default=0,
                   help="cap on tiles per persistent GEMM block (0 = auto: 8, the launcher picks the makespan-optimal "
                        "count under it; 1 = one block per tile)")
    p.add_argument("--min_bpc", type=int, default=0,
                   help="minimum blocks per CU of persistent GEMM grids (0 = auto: 2 with overlapping collectives)")
    p.add_argument("--wgrad_stream", action=argparse.BooleanOptionalAction, default=True,
                   help="N=1 fused path: weight-gradient GEMMs (fused SGD) on a second stream, concurrent with the "
                        "dgrads; the dispatcher fills each GEMM's tail with the other's blocks (0.5 %% faster in 5/5 "
                        "interleaved pairs, profiles/r2/wgrad_stream_ab_r2.log); --no-wgrad_stream = serial.  The "
                        "engine uses it only while a weight gradient has <= 4 tiles per CU (TrainConfig."
                        "wgrad_stream_max_tpc): D8192 (16 per CU) runs 131.5 ms concurrent vs 117.8 serial, the gated "
                        "Llama dims (7 per CU) 169.3 vs 167.0 (profiles/r3/wgrad_stream_tiles_per_cu_r3.txt, "
                        "gated_wgrad_stream_q16_r3.txt)")
    p.add_argument("--wgrad_stream_max_tpc", type=float, default=4.0,
                   help="use the weight-gradient stream only while a weight gradient has at most this many 256x256 "
                        "tiles per CU")
    p.add_argument("--data_overlap", action="store_true",
                   help="one-deep data pipeline: draw the next step's batch on a side stream under the current "
                        "backward (default: each batch on the compute stream at the start of its step).  The draw "
                        "co-runs with a backward GEMM and slows it: L8 flagship 30.18 / 30.63 vs 30.12 / 29.99 ms, "
                        "TP8 shard 0.630 vs 0.640 ms (profiles/r3/data_overlap_r3.txt)")
    p.add_argument("--no_relu_mask", action="store_true",
                   help="ReLU dgrad reads the bf16 activation instead of the forward's 1-bit mask")
    p.add_argument("--fp32_gemm", choices=["bf16x6", "mfma_f32"], default="bf16x6",
                   help="--dtype fp32 GEMMs: exact 3-way bf16 split on the bf16 MFMA kernels, or the fp32 MFMA kernel")
    p.add_argument("--master", choices=["split", "fp32"], default="split",
                   help="fp32 master weights of a bf16 run: split (bf16 working copy + int16 residual, exactly the "
                        "fp32 master, 4 B/param) or a separate fp32 buffer (6 B/param with the copy)")
    p.add_argument("--group_m_nt", type=int, default=4,
                   help="tiles per raster band of the NT-layout GEMMs")
    p.add_argument("--group_m_nn", type=int, default=8,
                   help="tiles per raster band of the NN-layout GEMMs")
    p.add_argument("--group_m_tn", type=int, default=4,
                   help="tiles per raster band of the TN-layout GEMMs")
    p.add_argument("--dist_first", action="store_true",
                   help="diagnostic: create the process group before the N=1 headline (as N>1 runs must)")
    p.add_argument("--force_comm", action="store_true",
                   help="exercise the RCCL DDP/FSDP path of the headline at N=1 (size-1 communicators)")
    p.add_argument("--zero_copy", action="store_true",
                   help="with --force_comm (ZeRO-2 headline at N=1): copying size-1 reduce-scatters / all-gathers (a "
                        "separate gradient shard, an all-gather sink) -- the zero_copy side entry as the headline")
    p.add_argument("--hw_queues", type=int, default=0,
                   help="GPU_MAX_HW_QUEUES for this run (HIP hardware queues per process; 0 = leave HIP's setting, "
                        "default 4).  Set before the first HIP call; self-launched ranks inherit it")
    p.add_argument("--no_queue_reserve", action="store_true",
                   help="do not reserve the compute stream's hardware queue at start (utils/streams.py)")
    p.add_argument("--diff_pairs", type=int, default=3,
                   help="communicating methods: interleaved pairs of (--diff_steps normal steps, --diff_steps steps with "
                        "every collective elided); exposed_ms_diff = median normal - median elided step time")
    p.add_argument("--diff_steps", type=int, default=4)
    p.add_argument("--elide_collectives", action="store_true",
                   help="diagnostic (not a valid measurement of the method): run every step with the collectives "
                        "elided, as the exposed_ms_diff reference steps do, e.g. to kernel-trace both variants")
    p.add_argument("--no_pair_wgrads", action="store_true",
                   help="run small-grid weight-gradient pairs (the MP / TP8 shard) as two split-K GEMMs instead of one "
                        "grouped launch")
    return p.parse_args(argv)


def mesh_of(method: str, n: int, tp_arg: int) -> tuple[str, int, int]:
    """(dp_mode, dp, tp) of a method on n ranks."""
    if method in ("ddp", "zero", "fsdp"):
        return method, n, 1
    if method == "tp":
        return "none", 1, n
    tp = tp_arg or min(n, 2)
    return "fsdp", n // tp, tp


def parallelism(method, n, dp, tp, world, force_comm) -> str:
    if world == 1 and not force_comm and method in ("ddp", "zero", "fsdp"):
        return "dp1"  # one device: no gradient collective, the optimizer is fused into the wgrad GEMMs
    return {"ddp": f"dp{n}", "zero": f"dp{n}-zero2", "fsdp": f"fsdp{n}", "tp": f"tp{n}",
            "hybrid": f"fsdp{dp}xtp{tp}"}[method] + ("-forcecomm" if world == 1 and force_comm else "")


def model_name(m: ModelConfig) -> str:
    return f"ffn-stack L{m.layers} D{m.D} F{m.F} {'swiglu-' if m.gated else ''}{m.act}"


def state_gib(eng) -> dict:
    """Per-rank persistent training state (GiB): fp32 master (+ optimizer moments), compute copy, grads."""
    g = lambda t: round(t.numel() * t.element_size() / 2**30, 3)  # noqa: E731
    key = "master_residual" if eng.split else "master_fp32"  # split: the fp32 master = working copy + int16 plane
    out = {key: round(eng.master_bytes / 2**30, 3), "compute_copy": 0.0 if eng.shared_copy else g(eng.copy),
           "grads": g(eng.grads)}
    if getattr(eng, "adam_m", None) is not None:
        out["adam_mv"] = round(2 * g(eng.adam_m), 3)
    return out


def destroy_mesh(mesh: Mesh) -> None:
    """Tear down this method's communicators (native ones and torch role process groups) so the next
    method's mesh does not hold stale RCCL resources."""
    import torch.distributed as dist

    torch_groups = [g for g in mesh.groups.values()
                    if isinstance(g, dist.ProcessGroup) and g is not dist.GroupMember.WORLD]
    mesh.destroy()
    if dist.is_initialized():
        dist.barrier()
        seen = set()
        for g in torch_groups:
            if id(g) not in seen:
                seen.add(id(g))
                dist.destroy_process_group(g)


def run_method(a, method: str, n: int, world: int, dev: torch.device, steps: int, warmup: int,
               force_comm: bool, model: ModelConfig, observe_steps: int = 0, headline: bool = False,
               windows: tuple = (0.0, 0.0, 0), fsdp_alias: bool = True, zero_alias: bool = True,
               min_bpc: int | None = None) -> dict:
    """Build the engine for ``method`` on ``n`` ranks, run ``warmup`` untimed + ``steps`` timed steps (+ the
    observed steps), return the method's record.  Collective over all ranks.

    ``windows`` = (min warm-up ms, min timed ms, max timed steps): the side-by-side methods' steady-state windows
    (the headline keeps the driver's exact step counts: (0, 0, 0)).  ``fsdp_alias`` False: FSDP at dp = 1 runs its
    gather / gradient rings and real (copying) size-1 collectives instead of aliasing the full buffers; ``zero_alias``
    False: ZeRO-2 at dp = 1 with a separate gradient shard and an all-gather sink (copying size-1 collectives).
    ``min_bpc``: overrides --min_bpc."""
    cpu = dev.type == "cpu"
    dp_mode, dp, tp = mesh_of(method, n, a.tp)
    cfg = TrainConfig(model=model, batch_size=a.batch_size, seq_len=a.seq_len, num_steps=steps, dtype=a.dtype,
                      grad_dtype=a.grad_dtype, optimizer=a.optimizer, dp_mode=dp_mode, dp=dp, tp=tp,
                      bucket_mb=a.bucket_mb, recompute=a.recompute, sequence_parallel=a.sequence_parallel,
                      data="device", force_comm=force_comm, comm_backend=a.comm,
                      force_tp_comm=force_comm and method in ("tp", "hybrid"),
                      side_optimizer=a.side_opt if headline else 0, tp_allreduce=a.tp_allreduce,
                      wgrad_layout=a.wgrad_layout, w2_storage=a.w2_storage,
                      relu_mask=not a.no_relu_mask, gemm_tiles_per_block=a.tpb, fp32_gemm=a.fp32_gemm,
                      gemm_min_bpc=a.min_bpc if min_bpc is None else min_bpc, master=a.master, wgrad_stream_max_tpc=a.wgrad_stream_max_tpc,
                      wgrad_stream=a.wgrad_stream and headline and not a.graph,
                      tp_transposed=os.environ.get("DLLM_TP_TRANSPOSED", "1") != "0", fsdp_alias=fsdp_alias,
                      zero_alias=zero_alias)
    mesh = Mesh.build(dp, tp, force=force_comm, comm_backend="torch" if cpu else a.comm,
                      device=None if cpu else dev)
    try:
        return _run_on_mesh(a, method, cfg, mesh, n, world, dev, steps, warmup, force_comm, model, observe_steps,
                            headline, windows)
    except BaseException:
        # error path (e.g. out of memory on one rank): abort this method's communicators, so they neither leak
        # into the next method nor block in a synchronising teardown against peers that moved on
        mesh.destroy(abort=True)
        raise


def _agree_max(x: float, world: int, dev) -> float:
    """The maximum of ``x`` over all ranks (every rank must take the same number of steps)."""
    if world <= 1:
        return x
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _run_on_mesh(a, method, cfg, mesh, n, world, dev, steps, warmup, force_comm, model, observe_steps, headline,
                 windows=(0.0, 0.0, 0)):
    cpu = dev.type == "cpu"
    sync = (lambda: None) if cpu else torch.cuda.synchronize
    dp, tp = cfg.dp, cfg.tp
    if not cpu:
        torch.cuda.reset_peak_memory_stats(dev)
    eng = FFNTrainer(cfg, mesh, dev)
    from dllm.models.ffn import init_ffn_params_device

    init_scale = "fan_in" if a.init_scale in ("auto", "fan_in") else float(a.init_scale)
    eng.load_full_params(init_ffn_params_device(model.D, model.F, model.layers, a.seed, dev, model.gated,
                                                scale=init_scale))
    sync()
    # --data_overlap: one-deep data pipeline, step s+1's batch drawn on a side stream under step s's backward
    data = DeviceMockData(cfg.tokens, model.D, cfg.torch_dtype, dev, overlap=a.data_overlap and not a.graph)
    seed_base = 10_000 * (mesh.dp_rank + 1)

    graphed = None
    if a.graph and headline:
        from dllm.utils.graphs import GraphedStep

        graphed = GraphedStep(eng, cfg.tokens, model.D)
    else:
        eng.before_backward = data.release
        data.bind_transposed(*eng.input_transposes())   # the NN layout's xᵀ / dyᵀ drawn with the batch

    def one_step(seed):
        old = comm.set_elide(True) if a.elide_collectives else None
        try:
            if graphed is not None:
                graphed.step(seed)
            else:
                x, dy = data.fill(seed, next_seed=seed + 1)
                eng.train_step(x, dy)
        finally:
            if old is not None:
                comm.set_elide(old)

    queues = None

    def queue_probe():
        # which streams share the compute stream's hardware queue; probes spin the GPU and synchronise, so this runs
        # after the FIRST warm-up step (every stream exists and has run), not between the warm-up and the timed steps:
        # an idle gap there lets the clock drop and the timed window would start cold (TP8 shard: 0.509 vs 0.485 ms)
        nonlocal queues
        if not cpu and a.backend == "nccl":
            # every stream of this method exists and has run by now: measure which share the compute stream's queue
            from dllm.utils.streams import queue_report

            sync()
            sides = {"wgrad": eng.wg_stream, "opt": getattr(eng, "opt_stream", None),
                     "fsdp": getattr(eng, "fsdp_stream", None), "data": getattr(data, "_stream", None)}
            queues = queue_report(dev, sides)
            if mesh.groups:
                # pairwise: role communicators' streams (identified at mesh build) and the side streams; conflicts =
                # any of them on the compute queue, or the FSDP gather and reduce-scatter on one queue
                from dllm.utils.streams import role_queue_report

                named = {r: mesh.role_streams.get(r) for r in mesh.groups if mesh.groups[r] is not None}
                named.update({k: v for k, v in sides.items() if v is not None})
                queues.update(role_queue_report(dev, named))

    min_warm_ms, min_timed_ms, max_steps = windows
    t_w = time.perf_counter()
    for i in range(warmup):
        one_step(seed_base + i)
        if i == 0:
            queue_probe()
    nwarm = warmup
    if min_warm_ms > 0 or min_timed_ms > 0:
        # steady-state windows (side methods): warm up on GPU time, not a step count -- the clock ramps over the first
        # ~50 ms of load -- in doubling batches of timed steps (first steps are slow: allocation, queue creation) until
        # the warm-up reaches min_warm_ms; the last batch's step time sizes the timed window (+20 % margin); every
        # rank agrees on every count
        sync()
        batch, step_ms = 1, float("inf")
        while True:
            t1 = time.perf_counter()
            for i in range(batch):
                one_step(seed_base + nwarm + i)
            sync()
            dt = _agree_max((time.perf_counter() - t1) * 1e3, world, dev)
            nwarm += batch
            if batch >= 2:   # the fastest multi-step batch: the first steps (allocation, queue creation) read slow
                step_ms = min(step_ms, dt / batch)
            if _agree_max((time.perf_counter() - t_w) * 1e3, world, dev) >= min_warm_ms and batch >= 2:
                break
            batch *= 2
        steps = max(steps, min(max_steps or steps, int(-(-1.2 * min_timed_ms // max(step_ms, 1e-3)))))
    warm_total_ms = _agree_max((time.perf_counter() - t_w) * 1e3, world, dev) if (min_warm_ms > 0 or min_timed_ms > 0) \
        else (time.perf_counter() - t_w) * 1e3
    if warmup == 0:
        queue_probe()
    if a.phases and headline and not cpu and graphed is None:
        eng.enable_phase_timing(True)
    sync()
    comm.barrier(device=dev)
    t0 = time.perf_counter()
    for i in range(steps):
        one_step(seed_base + nwarm + i)
    sync()
    comm.barrier(device=dev)
    el = time.perf_counter() - t0
    eng.check_health()
    phases = {k: round(v / steps, 3) for k, v in eng.phase_summary().items()} if (a.phases and headline) else None
    if world > 1:
        import torch.distributed as dist

        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ms = el / steps * 1e3
    rec = {"value": round(cfg.tokens * dp * steps / el, 1), "ms_per_step": round(ms, 3),
           "tflops_per_gpu": round(flops_per_step(cfg, tp=tp, recompute=cfg.recompute) / (ms / 1e3) / 1e12, 1),
           "peak_hbm_gib": 0.0 if cpu else round(torch.cuda.max_memory_allocated(dev) / 2**30, 2),
           # every weight of this rank's working copy (the split master's hi plane / the bf16 copy / the fp32 master)
           "finite": bool(torch.isfinite(eng.copy).all().item()),
           "init": init_scale,
           "master": "fp32 (split: bf16 working copy + int16 residual)" if eng.split else "fp32",
           "global_batch": a.batch_size * dp, "parallelism": parallelism(method, n, dp, tp, world, force_comm),
           "model": model_name(model), "steps": steps, "warmup": nwarm, "state_gib": state_gib(eng),
           "warmup_ms": round(warm_total_ms, 1), "timed_ms": round(el * 1e3, 1),
           "wgrad_stream": eng.wg_stream is not None,
           # small-grid weight gradients in one grouped launch / F-major activations on 224-row tiles (MP at tp 8)
           "pair_wgrads": bool(eng.pair_wgrads), "tp_transposed": bool(eng.tmode),
           "wgrad_nn": bool(eng.wgrad_nn), "wgrad_nn_w2": bool(eng.wgrad_nn_w2), "w2_transposed": bool(eng.w2s),
           # the ranks each role communicator actually spans (RCCL / gloo group sizes; {} = no collective)
           "comm_sizes": {role: g.size() for role, g in mesh.groups.items() if g is not None}}
    if eng.tp_ar_choice is not None:
        rec["tp_allreduce_choice"] = eng.tp_ar_choice
    if a.elide_collectives:
        rec["collectives_elided"] = True   # diagnostic run: not the method's step time
    if phases:
        rec["phase_ms_per_step"] = phases
    if queues is not None:
        rec["queues"] = queues
    communicates = bool(mesh.groups) or eng.tp_car is not None
    nxt = seed_base + nwarm + steps
    if observe_steps > 0 and communicates and not cpu and graphed is None:
        from dllm.utils.observe import CommObserver

        with CommObserver(dev, dict(mesh.groups)) as obs:
            for i in range(observe_steps):
                one_step(nxt + i)
        nxt += observe_steps
        rec["comm"] = obs.summary(observe_steps)
    if "comm" in rec and world == 1:
        # every collective a size-1 communicator that moved no data (aliased in place): the method's comm numbers say
        # nothing about collectives at N > 1
        c = rec["comm"]
        c["collectives_noop"] = bool(c.get("collectives_per_step")) and \
            c.get("noop_collectives_per_step") == c.get("collectives_per_step")
    if a.diff_pairs > 0 and a.diff_steps > 0 and communicates and graphed is None and not a.elide_collectives:
        # differential exposed communication: the same engine with its collectives elided (compute only), interleaved
        # with normal steps in this process; the difference of the medians is the step time the collectives add
        on, off = [], []
        # each segment >= ~100 ms of steps (sub-ms methods: short windows read the clock ramp, not the collectives)
        dsteps = max(a.diff_steps, min(max_steps or a.diff_steps, int(-(-100.0 // max(el * 1e3 / steps, 1e-3)))))
        for _ in range(a.diff_pairs):
            for elide, acc in ((False, on), (True, off)):
                old = comm.set_elide(elide)
                try:
                    sync()
                    comm.barrier(device=dev)
                    t1 = time.perf_counter()
                    for i in range(dsteps):
                        one_step(nxt + i)
                    sync()
                    comm.barrier(device=dev)
                    dt = time.perf_counter() - t1
                finally:
                    comm.set_elide(old)
                nxt += dsteps
                if world > 1:
                    import torch.distributed as dist

                    t = torch.tensor([dt], dtype=torch.float64, device=dev)
                    dist.all_reduce(t, op=dist.ReduceOp.MAX)
                    dt = float(t.item())
                acc.append(dt / dsteps * 1e3)
        med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
        c = rec.setdefault("comm", {})
        c["exposed_ms_diff"] = round(med(on) - med(off), 3)
        c["diff_step_ms"] = {"normal": [round(v, 3) for v in on], "collectives_elided": [round(v, 3) for v in off]}
        c["diff_steps"] = dsteps
    if eng.zero:
        eng.zero_sync_state()  # quiesce in-flight weight all-gathers before teardown
    sync()
    destroy_mesh(mesh)
    del eng, data, graphed
    gc.collect()
    if not cpu:
        torch.cuda.empty_cache()
    return rec


def data_note(init, finite: bool, overlap: bool = False) -> str:
    """The JSON ``data`` string.  Whether the data stayed finite is read from the run (``finite``: every weight of the
    working copy after the timed steps), never assumed: ``--init_scale 0.02`` overflows the flagship stack."""
    return ("synthetic (device Philox N(0,1) x, 0.1*N(0,1) dloss/dx, drawn every step" +
            (", the next batch on a side stream under the backward" if overlap else "") +
            f"; random-init weights, std {init}: " +
            ("finite data throughout" if finite else
             "NON-FINITE: the weights overflowed to inf / NaN during the run, the GEMMs ran on degenerate data") +
            ", see reference_init)")


SIDE_KEYS = ("value", "ms_per_step", "tflops_per_gpu", "peak_hbm_gib", "parallelism", "model", "global_batch",
             "steps", "warmup", "warmup_ms", "timed_ms", "finite", "init", "state_gib", "comm", "queues", "comm_sizes",
             "pair_wgrads", "tp_transposed", "wgrad_nn", "wgrad_nn_w2", "w2_transposed", "tp_allreduce_choice")


def main(argv=None) -> int:
    a = parse(argv)
    if a.hw_queues > 0:
        os.environ["GPU_MAX_HW_QUEUES"] = str(a.hw_queues)   # read by HIP at its first call, which is below
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    n = a.gpus or world
    if n != world:
        raise SystemExit(f"--gpus {n} but WORLD_SIZE={world}: the launcher started a different number of ranks")
    cpu = a.backend == "gloo"
    methods = [m for m in a.methods.split(",") if m and m != "none"]
    if not cpu:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
        if not a.no_queue_reserve:
            # before any process group / RCCL communicator / torch stream pool exists (utils/streams.py)
            from dllm.utils.streams import reserve_compute_queue

            reserve_compute_queue(torch.cuda.current_device())
    def init_dist():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        init_distributed("gloo" if a.backend == "gloo_gpu" else a.backend)

    # At N=1 the headline needs no process group: the side methods' one is created after it.  An RCCL communicator
    # that exists while the headline runs costs it 1.3-2.2 % (30.54-30.70 vs 30.04-30.14 ms interleaved,
    # profiles/r3/headline_rccl_init_order_r3.txt)
    if world > 1 or a.force_comm or a.dist_first:
        init_dist()
    diag_streams = []
    if os.environ.get("DLLM_DIAG_STREAMS") and not cpu:   # diagnostic: idle extra streams (count, priority)
        cnt, _, prio = os.environ["DLLM_DIAG_STREAMS"].partition(":")
        diag_streams = [torch.cuda.Stream(priority=int(prio or 0)) for _ in range(int(cnt))]
        for st in diag_streams:   # touch each so its HW queue is live
            with torch.cuda.stream(st):
                torch.zeros(1, device="cuda").add_(1)
        torch.cuda.synchronize()
    dev = torch.device("cpu") if cpu else torch.device("cuda", torch.cuda.current_device())
    if a.gemm_variant != "auto" and not cpu:
        from dllm.ops.gemm import set_bf16_variant

        set_bf16_variant(a.gemm_variant)
    if not cpu:
        from dllm.ops.gemm import set_group_m_nn, set_group_m_nt, set_group_m_tn, set_pair_wgrads

        set_group_m_nt(a.group_m_nt)
        set_group_m_nn(a.group_m_nn)
        set_group_m_tn(a.group_m_tn)
        set_pair_wgrads(not a.no_pair_wgrads)
    ffn = a.ffn_dim or (a.mp_ffn_dim if a.method == "tp" else 0)
    model = ModelConfig(model_size=a.model_size, ffn_dim=ffn, layers=a.layers, act=a.act, gated=a.gated)
    head = run_method(a, a.method, n, world, dev, a.steps, a.warmup, a.force_comm, model,
                      observe_steps=a.observe_steps, headline=True, zero_alias=not a.zero_copy)
    head_policy = None
    if not cpu:
        from dllm.ops.gemm import _POLICY

        head_policy = dict(_POLICY)
    ref_init = None
    if not cpu and not a.no_reference_init and a.init_scale in ("auto", "fan_in") and not model.gated:
        # the same headline run with the reference's 2e-2 init (diverges after the first update; see --init_scale)
        import copy as _copy

        a_ref = _copy.copy(a)
        a_ref.init_scale = "0.02"
        r = run_method(a_ref, a.method, n, world, dev, min(a.steps, 20), min(a.warmup, 5), a.force_comm, model,
                       headline=True)
        ref_init = {"init": 0.02, "ms_per_step": r["ms_per_step"], "value": r["value"], "finite": r["finite"],
                    "tflops_per_gpu": r["tflops_per_gpu"], "steps": r["steps"],
                    "note": "the reference's init scale: the stack overflows to inf / NaN after the first update and "
                            "the GEMMs then run on degenerate data (faster on MI355X: data-dependent power)"}
    if methods and not (world > 1 or a.force_comm or a.dist_first):
        init_dist()

    side: dict = {}
    import torch.distributed as dist

    def record(note: str = "") -> dict:
        rec = {
            "metric": METRIC, "value": head["value"], "unit": "tokens/s", "n_gpus": n,
            "world_size": dist.get_world_size() if dist.is_initialized() else 1, "comm_sizes": head["comm_sizes"],
            "launcher": "self" if os.environ.get("DLLM_SELF_LAUNCHED") else ("torchrun" if world > 1 else "none"),
            "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "default"),
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": head["ms_per_step"], "higher_is_better": True,
            "scaling": "strong" if a.method == "tp" else "weak", "vs_baseline": None, "dtype": a.dtype,
            "data": data_note(head.get("init"), head["finite"], a.data_overlap), "finite": head["finite"],
            "config": {"model": head["model"], "global_batch": head["global_batch"], "seq_len": a.seq_len,
                       "parallelism": head["parallelism"], "optimizer": a.optimizer, "grad_dtype": a.grad_dtype,
                       "master_weights": head.get("master", "fp32")},
            "tflops_per_gpu": head["tflops_per_gpu"],
            "mfu_dense": round(head["tflops_per_gpu"] / peak_tflops(a.dtype, a.fp32_gemm), 4),
            "peak_hbm_gib": head["peak_hbm_gib"], "state_gib": head["state_gib"],
            "comm_backend": a.comm, "hip_graph": bool(a.graph), "gemm_variant": a.gemm_variant,
            "tp_allreduce": a.tp_allreduce, "wgrad_stream": head.get("wgrad_stream", False),
            "pair_wgrads": head.get("pair_wgrads", False), "tp_transposed": head.get("tp_transposed", False),
            "wgrad_nn": head.get("wgrad_nn", False), "wgrad_nn_w2": head.get("wgrad_nn_w2", False),
            "w2_transposed": head.get("w2_transposed", False),
        }
        if head_policy is not None:
            rec["gemm_policy"] = head_policy   # raster bands, tiles per block, blocks per CU of the headline's GEMMs
        if ref_init is not None:
            rec["reference_init"] = ref_init
        for k in ("comm", "phase_ms_per_step", "queues", "collectives_elided"):
            if k in head:
                rec[k] = head[k]
        if side:
            rec["methods"] = dict(side)
            if world == 1:
                rec["methods_note"] = ("N=1: ddp/zero/fsdp/tp/hybrid run their collective code paths over size-1 "
                                       "communicators, which alias in place and move no data (comm.collectives_noop); "
                                       "fsdp_copy / zero_copy are FSDP / ZeRO-2 with real copying size-1 gathers / "
                                       "reduce-scatters (zero_copy at two GEMM blocks per CU, the N>1 policy); tp is the "
                                       "MP config (hidden 4096, FFN 14336, 1 layer); hybrid is the Llama-3-8B-dims "
                                       "SwiGLU stack (32 layers) on FSDP x TP; side methods are timed on steady-state "
                                       "windows (warmup_ms, timed_ms)")
        if a.force_comm:
            rec["note"] = "force_comm: headline collectives over size-1 RCCL communicators"
        if cpu:
            rec["note"] = f"CPU/gloo dry run with {world} ranks (plumbing only, not a measurement)"
        elif a.backend == "gloo_gpu":
            rec["note"] = (f"gloo_gpu rehearsal: {world} ranks on {torch.cuda.device_count()} GPU(s), gloo collectives "
                           "through the host (plumbing only, not a measurement)")
        if note:
            rec["note"] = (rec.get("note", "") + "; " + note).lstrip("; ")
        return rec

    printed = threading.Lock()
    done = {"printed": False}

    def emit(rec: dict) -> None:
        with printed:
            if done["printed"]:
                return
            done["printed"] = True
            if rank == 0:
                print(json.dumps(rec), flush=True)
                if a.json_out:
                    with open(a.json_out, "w") as f:
                        json.dump(rec, f)

    # The headline is measured; the side-by-side methods must not be able to lose it.  A side method that hangs
    # (e.g. a collective that never completes) is cut off at the deadline on every rank: rank 0 prints the line
    # with the methods finished so far, and each rank exits cleanly instead of waiting for the launcher's kill.
    current = {"m": None}

    def on_deadline() -> None:
        if not done["printed"]:
            side[current["m"] or "?"] = {"error": f"not finished within --side_deadline_s {a.side_deadline_s}"}
            rec = record(f"side method {current['m']} cut off at the deadline")
            rec["side_cut_off"] = current["m"] or "?"  # machine-readable: the headline is valid, a side method is not
            emit(rec)
        sys.stdout.flush()
        # the headline line is printed and valid: exit 0 so drivers keep it; side_cut_off marks the cut-off method
        os._exit(0)

    watchdog = None
    if methods and a.side_deadline_s > 0:
        watchdog = threading.Timer(a.side_deadline_s, on_deadline)
        watchdog.daemon = True
        watchdog.start()
    if world == 1 and "fsdp" in methods and "fsdp_copy" not in methods:
        # N=1: FSDP's size-1 collectives alias the full buffers and move nothing; fsdp_copy runs the dp > 1 ring
        # schedule with real (copying) RCCL gathers / reduce-scatters, so its exposed_ms_diff measures collectives
        methods.insert(methods.index("fsdp") + 1, "fsdp_copy")
    if world == 1 and "zero" in methods and "zero_copy" not in methods:
        # N=1 proxy of the N>1 headline schedule: ZeRO-2 with copying size-1 RCCL reduce-scatters
        # (gradients -> a separate shard) and all-gathers (the updated copy -> a sink), at the N>1 grid policy of two
        # persistent blocks per CU
        methods.insert(methods.index("zero") + 1, "zero_copy")
    for m in methods:
        current["m"] = m
        mm = model
        if m == "tp":
            mm = ModelConfig(model_size=a.model_size, ffn_dim=a.mp_ffn_dim, layers=a.mp_layers, act=a.act,
                             gated=a.gated)
        elif m == "hybrid":
            mm = ModelConfig(model_size=a.model_size, ffn_dim=a.llama_ffn_dim, layers=a.llama_layers, act="silu",
                             gated=True)
        try:
            base = {"fsdp_copy": "fsdp", "zero_copy": "zero"}.get(m, m)
            r = run_method(a, base, n, world, dev, a.method_steps or min(a.steps, 10),
                           min(a.warmup, 3), force_comm=(world == 1), model=mm, observe_steps=a.observe_steps,
                           windows=(a.side_warmup_ms, a.side_timed_ms, a.side_max_steps),
                           fsdp_alias=m != "fsdp_copy", zero_alias=m != "zero_copy",
                           min_bpc=(a.min_bpc or 2) if m == "zero_copy" else None)
        except (ValueError, RuntimeError) as e:
            # a side measurement must not cost the headline line (a config / memory error raises on every
            # rank alike; a hang is cut off by the deadline above)
            side[m] = {"error": f"{type(e).__name__}: {e}"[:300]}
            if not cpu:
                torch.cuda.empty_cache()
            continue
        side[m] = {k: r[k] for k in SIDE_KEYS if k in r}
    current["m"] = None
    emit(record())
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
