"""Flagship benchmark: FFN-stack training throughput (whole-node tokens/s) on MI355X.

Metric/config from BASELINE.json: "FFN tokens/sec (whole node) at hidden=4096 for DDP/FSDP/MP, 1/2/4/8
MI355X" on the 8-layer hidden=4096 FFN stack (FFN = 4·hidden = 16384, ReLU, as train_ffns.py:361),
batch 8 × seq 1024 = 8192 tokens per rank per step, bf16 compute with fp32 master weights, SGD (the
reference optimizer, train_ffns.py:172), random-init weights and synthetic device-generated data.

    python bench.py --gpus N --steps K --warmup W            # N=1 in-process
    torchrun --nproc-per-node N bench.py --gpus N ...          # one rank per GPU over RCCL/xGMI

Each timed step is the full training step: device mock-data generation, forward, backward (all weight
and input gradients except the unused layer-0 input grad), gradient communication and the optimizer
update.  Default parallelism for N>1 is data parallel with ZeRO-2 sharding (bf16 gradient reduce-scatter,
fp32 master weights sharded 1/N, bf16 weight all-gather); with N=1 there is no gradient collective and
the SGD update is fused into the weight-gradient GEMM epilogues.  K steps are bracketed by cuda synchronize + barrier on both sides; the max over ranks is
reported; rank 0 prints ONE JSON line.  Weak scaling: every rank processes 8192 tokens per step under
DDP/FSDP (global batch = 8·N sequences); ``--method tp`` shards each layer over the GPUs instead
(tokens per step fixed: strong scaling).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

import dllm  # noqa: F401
from dllm.parallel import comm
from dllm.parallel.engine import FFNTrainer
from dllm.parallel.mesh import Mesh, init_distributed
from dllm.utils.config import ModelConfig, TrainConfig
from dllm.utils.data import DeviceMockData
from dllm.utils.metrics import PEAK_TFLOPS, flops_per_step

METRIC = "FFN tokens/sec (whole node) at hidden=4096 for DDP/FSDP/MP, 1/2/4/8 MI355X"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=0)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--method", choices=["ddp", "zero", "fsdp", "tp", "hybrid"], default="zero",
                   help="zero = data parallel with ZeRO-2 (bucketed reduce-scatter overlapped with the backward, "
                        "1/N sharded optimizer, async all-gather of the bf16 weights overlapped with the next "
                        "forward); ddp = bucketed all-reduce + full optimizer per rank")
    p.add_argument("--tp", type=int, default=0, help="TP degree for --method hybrid")
    p.add_argument("--model_size", type=int, default=4096)
    p.add_argument("--ffn_dim", type=int, default=0)
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
                   help="weight init std: a number, 'fan_in' (1/sqrt(fan_in) per matrix), or 'auto' = the "
                        "reference's 2e-2 for plain FFN stacks and fan_in for gated (SwiGLU) stacks, which "
                        "overflow with 2e-2 once deep (no norms/residuals in this model)")
    p.add_argument("--json_out", default="")
    p.add_argument("--comm", choices=["torch", "native"], default="torch",
                   help="role communicators: torch ProcessGroupNCCL or the native C++ RCCL layer")
    p.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                   help="gloo = CPU dry run of the multi-rank path (tests; tiny dims)")
    p.add_argument("--graph", action="store_true",
                   help="capture the whole step (data + fwd + bwd + fused SGD) in a HIP graph (N=1 path)")
    p.add_argument("--side_opt", type=int, default=0,
                   help="N=1: store wgrads and run SGD on a side stream over this many workgroups (0 = fuse the "
                        "update into the wgrad GEMM epilogue)")
    p.add_argument("--phases", action="store_true",
                   help="also report per-phase GPU time (forward / backward / optimizer tail) from HIP events")
    p.add_argument("--tp_allreduce", choices=["rccl", "custom"], default="rccl",
                   help="TP activation all-reduce: RCCL, or the custom two-shot xGMI peer all-reduce (csrc/car.hip)")
    p.add_argument("--gemm_variant", default="auto",
                   choices=["auto", "2stage", "8phase", "8phase_stagger", "4phase_stagger"],
                   help="bf16 GEMM main-loop schedule (auto = 8-phase staggered when K % 128 == 0)")
    p.add_argument("--lib_plain_nt", action="store_true",
                   help="run the plain forward GEMM y = a·W2ᵀ (no epilogue) on hipBLASLt; all fused GEMMs stay native")
    p.add_argument("--tpb", type=int, default=0,
                   help="tiles per persistent 8-phase GEMM block (0 = auto: 2, or 1 for gated stacks; 1 = off)")
    p.add_argument("--wgrad_stream", action="store_true",
                   help="N=1: weight-gradient GEMMs (fused SGD) on a second stream, concurrent with the dgrads")
    p.add_argument("--no_relu_mask", action="store_true",
                   help="ReLU dgrad reads the bf16 activation instead of the forward's 1-bit mask")
    p.add_argument("--force_comm", action="store_true",
                   help="exercise the RCCL DDP/FSDP path at N=1 (size-1 communicators, unfused optimizer)")
    return p.parse_args()


def main() -> int:
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    n = a.gpus or world
    if n != world:
        raise SystemExit(f"--gpus {n} but WORLD_SIZE={world}: launch N>1 with torchrun")
    cpu = a.backend == "gloo"
    if world > 1 or a.force_comm:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        init_distributed(a.backend)
    elif not cpu:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dev = torch.device("cpu") if cpu else torch.device("cuda", torch.cuda.current_device())
    sync = (lambda: None) if cpu else torch.cuda.synchronize

    if a.method == "ddp":
        dp_mode, dp, tp = "ddp", n, 1
    elif a.method == "zero":
        dp_mode, dp, tp = "zero", n, 1
    elif a.method == "fsdp":
        dp_mode, dp, tp = "fsdp", n, 1
    elif a.method == "tp":
        dp_mode, dp, tp = "none", 1, n
    else:
        tp = a.tp or min(n, 2)
        dp_mode, dp = "fsdp", n // tp
    if a.gemm_variant != "auto" and not cpu:
        from dllm.ops.gemm import set_bf16_variant

        set_bf16_variant(a.gemm_variant)
    if a.lib_plain_nt:
        from dllm.ops.gemm import set_library_plain_nt

        set_library_plain_nt(True)
    m = ModelConfig(model_size=a.model_size, ffn_dim=a.ffn_dim, layers=a.layers, act=a.act, gated=a.gated)
    cfg = TrainConfig(model=m, batch_size=a.batch_size, seq_len=a.seq_len, num_steps=a.steps, dtype=a.dtype,
                      grad_dtype=a.grad_dtype, optimizer=a.optimizer, dp_mode=dp_mode, dp=dp, tp=tp,
                      bucket_mb=a.bucket_mb, recompute=a.recompute, sequence_parallel=a.sequence_parallel,
                      data="device", force_comm=a.force_comm, comm_backend=a.comm, side_optimizer=a.side_opt, tp_allreduce=a.tp_allreduce,
                      relu_mask=not a.no_relu_mask, gemm_tiles_per_block=a.tpb,
                      wgrad_stream=a.wgrad_stream)
    mesh = Mesh.build(dp, tp, force=a.force_comm, comm_backend="torch" if cpu else a.comm,
                      device=None if cpu else dev)
    eng = FFNTrainer(cfg, mesh, dev)
    from dllm.models.ffn import init_ffn_params_device

    init_scale = ("fan_in" if m.gated else 2e-2) if a.init_scale == "auto" else (
        a.init_scale if a.init_scale == "fan_in" else float(a.init_scale))
    eng.load_full_params(init_ffn_params_device(m.D, m.F, m.layers, a.seed, dev, m.gated, scale=init_scale))
    sync()
    data = DeviceMockData(cfg.tokens, m.D, cfg.torch_dtype, dev)
    seed_base = 10_000 * (mesh.dp_rank + 1)

    graphed = None
    if a.graph:
        from dllm.utils.graphs import GraphedStep

        graphed = GraphedStep(eng, cfg.tokens, m.D)

    def one_step(seed):
        if graphed is not None:
            graphed.step(seed)
        else:
            x, dy = data.fill(seed)
            eng.train_step(x, dy)

    for i in range(a.warmup):
        one_step(seed_base + i)
    if a.phases and not cpu and graphed is None:
        eng.enable_phase_timing(True)
    sync()
    comm.barrier(device=dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        one_step(seed_base + a.warmup + i)
    sync()
    comm.barrier(device=dev)
    el = time.perf_counter() - t0
    phases = {k: round(v / a.steps, 3) for k, v in eng.phase_summary().items()} if a.phases else None
    if world > 1:
        import torch.distributed as dist

        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ms = el / a.steps * 1e3
    tokens_global = cfg.tokens * dp
    value = tokens_global * a.steps / el
    tflops = flops_per_step(cfg, tp=tp, recompute=cfg.recompute) / (ms / 1e3) / 1e12
    finite = bool(torch.isfinite(eng.master[:1024]).all().item())
    peak_gib = 0.0 if cpu else torch.cuda.max_memory_allocated(dev) / 2**30
    if eng.zero:
        eng.zero_sync_state()  # quiesce in-flight weight all-gathers before teardown
    par = {"ddp": f"dp{n}", "zero": f"dp{n}-zero2", "fsdp": f"fsdp{n}", "tp": f"tp{n}",
           "hybrid": f"fsdp{dp}xtp{tp}"}[a.method]
    if world == 1 and not a.force_comm and a.method in ("ddp", "zero", "fsdp"):
        par = "dp1"  # one device: no gradient collective, the optimizer is fused into the wgrad GEMMs
    rec = {
        "metric": METRIC, "value": round(value, 1), "unit": "tokens/s", "n_gpus": 0 if cpu else n, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
        "scaling": "strong" if a.method == "tp" else "weak", "vs_baseline": None, "dtype": a.dtype,
        "data": "synthetic (device Philox N(0,1) x, 0.1*N(0,1) dloss/dx; random-init weights)",
        "config": {"model": f"ffn-stack L{m.layers} D{m.D} F{m.F} {'swiglu-' if m.gated else ''}{m.act}",
                   "global_batch": a.batch_size * dp, "seq_len": a.seq_len, "parallelism": par,
                   "optimizer": a.optimizer, "grad_dtype": a.grad_dtype, "master_weights": "fp32",
                   "init_scale": init_scale},
        "tflops_per_gpu": round(tflops, 1), "mfu_dense": round(tflops / PEAK_TFLOPS[a.dtype], 4),
        "peak_hbm_gib": round(peak_gib, 2), "finite": finite, "comm": a.comm, "hip_graph": bool(a.graph),
        "plain_nt_gemm": "hipblaslt" if a.lib_plain_nt else "native", "gemm_variant": a.gemm_variant,
        "gemm_tiles_per_block": a.tpb or ("auto: 1" if m.gated else "auto: 2"), "relu_mask": eng.masks is not None,
        "wgrad_stream": eng.wg_stream is not None,
        "tp_allreduce": a.tp_allreduce,
    }
    if phases:
        rec["phase_ms_per_step"] = phases
    if a.force_comm:
        rec["note"] = "force_comm: DDP/FSDP collectives over size-1 RCCL communicators"
    if cpu:
        rec["note"] = f"CPU/gloo dry run with {world} ranks (plumbing only, not a measurement)"
    if rank == 0:
        print(json.dumps(rec), flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                json.dump(rec, f)
    import torch.distributed as dist

    if dist.is_initialized():
        dist.barrier()
        mesh.destroy()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
