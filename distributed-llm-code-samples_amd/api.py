"""Reference-compatible functional API.

The module-level functions of the reference's ``train_ffns.py`` keep their names, signatures and
return structures here, so a script written against the reference runs by switching its imports:

    from dllm.api import init_tlayer_ffn, mock_data, train_1gpu, train_ddp, train_fsdp, train_tp

What runs underneath is this framework's:

* the primitives (``linear_fwd``, ``t_linear_bkwd``, ``tlayer_ffn_*``) go through ``ops.gemm`` — the
  gfx950 MFMA kernels for HIP tensors (fused ReLU / ReLU-mask epilogues), the torch oracle for CPU
  tensors;
* the trainers (``train_*``) run the unified engine (``parallel/engine.py``) over RCCL, one process per
  GPU (gloo on CPU-only hosts), and return the trained ``list[L]`` of ``[W1 [F,D], W2 [D,F]]`` fp32
  tensors on ``cuda:0`` (CPU without a GPU), like the reference (:116, :193, :287, :338);
* the ``train_process_*`` worker bodies run inside an already initialised process group
  (``init_process``) and write the result back into the tensors they were given, like the reference's
  IPC-shared in-place updates (:172, :259, :312).

Reference line numbers below are ``train_ffns.py``.
"""
from __future__ import annotations

import functools
import os

import torch
import torch.distributed as dist

from .models.ffn import init_linear_layer  # noqa: F401  (re-export, :35-36)
from .ops.activations import act_fwd, relu_bkwd_
from .ops.gemm import gemm
from .utils.config import DLOSS_DX_COEF, LR, ModelConfig, TrainConfig  # noqa: F401
from .utils.data import reference_mock_data

__all__ = [
    "LR", "DLOSS_DX_COEF", "nGPUs", "init_linear_layer", "init_tlayer_ffn", "linear_fwd", "t_linear_bkwd",
    "t_relu_fwd", "t_relu_bkwd_", "tlayer_ffn_fwd", "tlayer_ffn_bkwd", "tlayers_ffn_fwd", "tlayers_ffn_bkwd",
    "mock_data", "train_1gpu", "train_ddp", "train_fsdp", "train_tp", "train_zero", "init_process",
    "torch_profile_rank_0", "train_process_ddp", "train_process_fsdp", "train_process_tp",
]

nGPUs = torch.cuda.device_count()  # :25 (the reference refuses exactly one GPU; here any count works)


# --------------------------------------------------------------------------------------------------
# parameters and primitives (:35-70)
# --------------------------------------------------------------------------------------------------
def init_tlayer_ffn(emb_dim: int, ffn_dim: int, gen: torch.Generator | None = None) -> list[torch.Tensor]:
    """``[W1 [ffn, emb], W2 [emb, ffn]]``, drawn in that order (:38-39)."""
    return [init_linear_layer(emb_dim, ffn_dim, gen), init_linear_layer(ffn_dim, emb_dim, gen)]


def linear_fwd(layer_params: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """``x · Wᵀ`` (:41-42) — the NT GEMM."""
    return gemm(x.contiguous(), layer_params.contiguous(), "nt")


def t_linear_bkwd(dloss_dx: torch.Tensor, layer_params: torch.Tensor, x: torch.Tensor):
    """``(dW, dx) = (dyᵀ·x, dy·W)`` (:44-45) — the TN wgrad and NN dgrad GEMMs."""
    dy = dloss_dx.contiguous()
    return gemm(dy, x.contiguous(), "tn"), gemm(dy, layer_params.contiguous(), "nn")


def t_relu_fwd(x: torch.Tensor) -> torch.Tensor:
    """``where(x <= 0, 0, x)`` (:47-48)."""
    return act_fwd("relu", x)


def t_relu_bkwd_(dloss_dx: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """In-place ReLU backward mask (:50-52)."""
    return relu_bkwd_(dloss_dx, x)


def tlayer_ffn_fwd(layer_params, x: torch.Tensor) -> torch.Tensor:
    """``ReLU(x·W1ᵀ)·W2ᵀ`` (:54-58); the ReLU is fused into the first GEMM's epilogue."""
    w1, w2 = (p.contiguous() for p in layer_params)
    a = gemm(x.contiguous(), w1, "nt", epi="act", act="relu")
    return gemm(a, w2, "nt")


def tlayer_ffn_bkwd(dloss_dx: torch.Tensor, layer_params, x: torch.Tensor):
    """Backward of one layer from its saved input, recomputing the activation like the reference
    (:61-70).  Returns ``(dx, (dW1, dW2))``.  The ReLU mask is fused into the ``da`` dgrad epilogue
    (``ReLU(h) > 0`` iff ``h > 0``, so the recomputed activation serves as the mask)."""
    w1, w2 = (p.contiguous() for p in layer_params)
    x, dy = x.contiguous(), dloss_dx.contiguous()
    a = gemm(x, w1, "nt", epi="act", act="relu")           # recompute (:63, :66)
    dw2 = gemm(dy, a, "tn")                                  # dW2 = dyᵀ·a
    da = gemm(dy, w2, "nn", epi="dact", act="relu", aux=a)   # da = (dy·W2) ⊙ [h > 0]
    dw1 = gemm(da, x, "tn")                                  # dW1 = daᵀ·x
    dx = gemm(da, w1, "nn")                                  # dx = da·W1
    return dx.reshape(x.shape), (dw1, dw2)


def tlayers_ffn_fwd(layers_params, x: torch.Tensor, before_comms_hook=None):
    """Stack forward; returns ``(y, acts)`` with every layer's input saved (:72-81).
    ``before_comms_hook(handle) -> handle`` runs before each layer (unused by the reference's callers)."""
    y, acts, handle = x, [], None
    for lp in layers_params:
        acts.append(y)
        if before_comms_hook is not None:
            handle = before_comms_hook(handle)
        y = tlayer_ffn_fwd(lp, y)
    return y, acts


def tlayers_ffn_bkwd(dloss_dx: torch.Tensor, layers_params, acts, after_comms_hook=None):
    """Stack backward in reverse layer order; returns the per-layer grads and the hooks' handles in
    forward order (:83-94).  ``after_comms_hook((dW1, dW2))`` runs as soon as a layer's grads exist."""
    g, grads, handles = dloss_dx, [], []
    for i in reversed(range(len(layers_params))):
        g, dp = tlayer_ffn_bkwd(g, layers_params[i], acts[i])
        grads.append(dp)
        handles.append(after_comms_hook(dp) if after_comms_hook is not None else None)
    return list(reversed(grads)), list(reversed(handles))


def mock_data(seeds, batch_size: int, model_size: int):
    """The reference data stream (:144-151): per seed, ``x = randn(T, D)`` then ``0.1·randn(T, D)``."""
    return reference_mock_data(seeds, batch_size, model_size)


# --------------------------------------------------------------------------------------------------
# trainers (:101-116, :174-193, :262-287, :315-338)
# --------------------------------------------------------------------------------------------------
def _backend_and_ranks() -> tuple[str, int]:
    if torch.cuda.is_available():
        return "nccl", max(torch.cuda.device_count(), 1)
    return "gloo", int(os.environ.get("DLLM_CPU_RANKS", "2"))


def _logical(layers_params) -> list[dict]:
    out = []
    for lp in layers_params:
        w1, w2 = lp[0], lp[1]
        out.append({"w1": w1.detach().float().cpu().contiguous(), "w2": w2.detach().float().cpu().contiguous()})
    return out


def _run(method: int, layers_params, seeds, batch_size: int, model_size: int, nprocs: int | None = None,
         port: int | None = None, **train_kw) -> list[list[torch.Tensor]]:
    from .parallel.launch import spawn

    backend, n = _backend_and_ranks()
    if nprocs:
        n = nprocs
    ranks = 1 if method == 1 else n
    params = _logical(layers_params)
    D = params[0]["w1"].shape[1]
    F = params[0]["w1"].shape[0]
    if D != model_size:
        raise ValueError(f"model_size {model_size} does not match W1 {tuple(params[0]['w1'].shape)}")
    seeds = torch.as_tensor(seeds, dtype=torch.int64)
    cfg = TrainConfig(model=ModelConfig(model_size=D, ffn_dim=F, layers=len(params)), batch_size=1,
                      seq_len=int(batch_size), num_steps=len(seeds), data="cpu_compat", **train_kw)
    opts = {"params": params, "seeds": seeds.tolist(), "return_params": True, "return_full": True,
            "tp": ranks}
    port = port or 29500 + 17 * method + (os.getpid() % 1000)
    rec = spawn(ranks, cfg, method, backend, port, opts)
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    return [[p["w1"].to(dev), p["w2"].to(dev)] for p in rec["params"]]


def train_1gpu(layers_params, seeds, batch_size, model_size, port=None, **train_kw):
    """Single device, sequential steps (:101-116)."""
    return _run(1, layers_params, seeds, batch_size, model_size, None, port, **train_kw)


def train_ddp(layers_params, seeds, batch_size, model_size, nprocs=None, port=None, **train_kw):
    """Data parallel, seeds striped over ranks, summed gradients (:174-193)."""
    return _run(2, layers_params, seeds, batch_size, model_size, nprocs, port, **train_kw)


def train_fsdp(layers_params, seeds, batch_size, model_size, nprocs=None, port=None, **train_kw):
    """FSDP (ZeRO-3 + DP), dim-0 row shards (:262-287)."""
    return _run(3, layers_params, seeds, batch_size, model_size, nprocs, port, **train_kw)


def train_tp(layers_params, seeds, batch_size, model_size, nprocs=None, port=None, **train_kw):
    """Tensor ("model") parallel, W1 column / W2 row split, replicated data (:315-338)."""
    return _run(4, layers_params, seeds, batch_size, model_size, nprocs, port, **train_kw)


def train_zero(layers_params, seeds, batch_size, model_size, nprocs=None, port=None, **train_kw):
    """ZeRO-2 data parallel (extension): same results as ``train_ddp``."""
    return _run(6, layers_params, seeds, batch_size, model_size, nprocs, port, **train_kw)


# --------------------------------------------------------------------------------------------------
# process-level entry points (:121-141, :156-172, :197-259, :290-312)
# --------------------------------------------------------------------------------------------------
def init_process(rank, layers_params, seeds, batch_size, model_size, fn, world_size=None, backend=None):
    """Rendezvous at 127.0.0.1 and run ``fn(rank, layers_params, seeds, batch_size, model_size)`` (:121-127)."""
    from .parallel.mesh import init_distributed

    be = backend or ("nccl" if torch.cuda.is_available() else "gloo")
    world = world_size or int(os.environ.get("WORLD_SIZE", 0)) or max(nGPUs, 1)
    init_distributed(be, rank, world, "127.0.0.1", int(os.environ.get("MASTER_PORT", "29500")))
    return fn(rank, layers_params, seeds, batch_size, model_size)


class torch_profile_rank_0:  # noqa: N801  (reference name, :129-141)
    """Decorator: run the worker under ``torch.profiler`` (CPU + GPU activities, shapes, stacks) and export
    rank 0's trace to ``trace_profiler_trace.json``.  A picklable class instead of the reference's
    ``global`` wrapper, so it survives ``spawn`` and can wrap several functions."""

    def __init__(self, func, path: str = "trace_profiler_trace.json"):
        functools.update_wrapper(self, func)
        self.func, self.path = func, path

    def __call__(self, *args, **kwargs):
        from torch.profiler import ProfilerActivity, profile

        acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])
        with profile(activities=acts, record_shapes=True, with_stack=True) as prof:
            out = self.func(*args, **kwargs)
        if args and args[0] == 0:
            prof.export_chrome_trace(self.path)
            print("Profiler exported")
        return out


def _gather_cat(t: torch.Tensor, dim: int) -> torch.Tensor:
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t.contiguous())
    return torch.cat(parts, dim=dim)


def _worker(method: int, local_rank: int, layers_params, seeds, batch_size: int, model_size: int,
            shard_dims=None) -> None:
    from .parallel.engine import FFNTrainer
    from .parallel.launch import METHOD_MESH
    from .parallel.mesh import Mesh
    from .utils.data import make_data

    n = dist.get_world_size()
    on_gpu = dist.get_backend() == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")
    comm_dev = dev  # collectives of the set-up phase run on the backend's device
    full = []
    for lp in layers_params:
        w1, w2 = lp[0].to(comm_dev).float(), lp[1].to(comm_dev).float()
        if shard_dims is not None:  # the rank holds shards: rebuild the logical tensors
            w1, w2 = _gather_cat(w1, shard_dims[0]), _gather_cat(w2, shard_dims[1])
        full.append({"w1": w1, "w2": w2})
    dp_mode, dp, tp = METHOD_MESH[method](n, {"tp": n})
    D, F = full[0]["w1"].shape[1], full[0]["w1"].shape[0]
    cfg = TrainConfig(model=ModelConfig(model_size=D, ffn_dim=F, layers=len(full)), batch_size=1,
                      seq_len=int(batch_size), num_steps=len(seeds), data="cpu_compat", dp_mode=dp_mode, dp=dp, tp=tp)
    mesh = Mesh.build(dp, tp, device=dev if on_gpu else None)
    eng = FFNTrainer(cfg, mesh, dev)
    eng.load_full_params(full)
    # ``seeds`` are already this rank's own: the reference's drivers hand each DDP/FSDP worker its stripe
    # (cpus_seeds[rank], :182, :273) and every TP worker all seeds (:324)
    mine = torch.as_tensor(seeds, dtype=torch.int64)
    data = make_data("cpu_compat", cfg.tokens, D, cfg.torch_dtype, dev)
    order = mine.tolist()
    for s in order[:data.depth]:
        data.prefetch(int(s))
    for i, s in enumerate(order):
        x, dy = data.fill(int(s), next_seed=order[i + data.depth] if i + data.depth < len(order) else None)
        eng.train_step(x, dy)
    res = eng.local_params()  # full over dp (FSDP gathers), this rank's TP shard
    r = dist.get_rank()
    with torch.no_grad():
        for lp, p in zip(layers_params, res):
            w1, w2 = p["w1"], p["w2"]
            if method == 3:  # FSDP: the caller holds dim-0 row shards
                w1 = w1.chunk(n, dim=0)[r]
                w2 = w2.chunk(n, dim=0)[r]
            lp[0].copy_(w1.to(lp[0].device, lp[0].dtype))
            lp[1].copy_(w2.to(lp[1].device, lp[1].dtype))
    mesh.destroy()


def train_process_ddp(local_rank, layers_params, seeds, batch_size, model_size):
    """DDP worker (:156-172): full replicas in, trained replicas written back in place."""
    _worker(2, local_rank, layers_params, seeds, batch_size, model_size)


def train_process_fsdp(local_rank, layers_params, seeds, batch_size, model_size):
    """FSDP worker (:197-259): this rank's dim-0 row shards in, trained shards written back in place."""
    _worker(3, local_rank, layers_params, seeds, batch_size, model_size, shard_dims=(0, 0))


def train_process_tp(local_rank, layers_params, seeds, batch_size, model_size):
    """TP worker (:290-312): W1 dim-0 / W2 dim-1 shards in, trained shards written back in place."""
    _worker(4, local_rank, layers_params, seeds, batch_size, model_size, shard_dims=(0, 1))
