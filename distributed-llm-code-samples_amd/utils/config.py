"""Run configuration: a superset of the reference CLI (train_ffns.py:343-350).

Reference flags keep their short/long names and defaults; north-star extras are added with defaults
that reproduce the reference semantics (ReLU, FFN = 4·D, SGD, LR = 1e-5, summed DP gradients).
"""
from __future__ import annotations

import argparse
import dataclasses
from dataclasses import dataclass

import torch

LR = 1e-5            # train_ffns.py:29
DLOSS_DX_COEF = 0.1  # train_ffns.py:30
INIT_SCALE = 2e-2    # train_ffns.py:35
SEED_RANGE = 100_000  # train_ffns.py:360
METHODS = {0: "all", 1: "1gpu", 2: "ddp", 3: "fsdp", 4: "tp", 5: "hybrid", 6: "zero"}


@dataclass
class ModelConfig:
    model_size: int = 4              # D  (-d)
    ffn_dim: int = 0                 # F; 0 -> 4·D (train_ffns.py:361)
    layers: int = 1                  # L  (-l)
    act: str = "relu"                # relu | silu | gelu
    gated: bool = False              # SwiGLU-style W1/W3 gate (Llama FFN)

    @property
    def F(self) -> int:
        return self.ffn_dim or 4 * self.model_size

    @property
    def D(self) -> int:
        return self.model_size

    def num_params(self) -> int:
        per = (3 if self.gated else 2) * self.D * self.F
        return per * self.layers


@dataclass
class TrainConfig:
    model: ModelConfig = dataclasses.field(default_factory=ModelConfig)
    batch_size: int = 8              # -bs
    seq_len: int = 1024              # -n
    num_steps: int = 1               # -s
    random_seed: int = 0             # -r (0 = unseeded, train_ffns.py:355-358)
    dtype: str = "fp32"              # compute dtype: fp32 (reference parity) | bf16
    grad_dtype: str = "fp32"         # dtype of gradients / gradient collectives
    optimizer: str = "sgd"           # sgd (reference) | adam
    lr: float = LR
    adam_b1: float = 0.9
    adam_b2: float = 0.95
    adam_eps: float = 1e-8
    weight_decay: float = 0.0
    dp_mode: str = "none"            # none | ddp | zero (ZeRO-2: sharded optimizer) | fsdp (ZeRO-3)
    dp: int = 1
    tp: int = 1
    sequence_parallel: bool = False  # Megatron SP for the TP path (RS/AG over T instead of AR)
    recompute: str = "none"          # none (save activations) | full (reference: recompute h in bwd)
    bucket_mb: float = 0.0           # DDP bucket cap; 0 = one bucket per weight tensor
    data: str = "device"             # device (Philox on GPU) | cpu_compat (reference CPU generator)
    skip_input_grad: bool = True     # layer-0 dx is never consumed (reference computes it, :68)
    separate_streams: bool = True    # one communicator/stream per comm role
    tp_overlap: bool = True          # overlap the TP dx all-reduce with the dW2 / dW1 GEMMs
    tp_chunks: int = 4               # TP forward: split T into this many row chunks; chunk i's y all-reduce
                                     # runs while chunk i+1 computes, and the next layer's chunk i starts as
                                     # soon as that one all-reduce is done (1 = one all-reduce per layer)
    relu_mask: bool = True           # ReLU: the dgrad reads a 1-bit activation mask written by the forward
                                     # GEMM instead of the bf16 activation (GPU, 8-phase kernel shapes)
    # GPU, F/tp a multiple of 224 whose 224-row tile grid fills the chip better (the MP config at tp = 8): keep activations as [F, T] and W2 as W2ᵀ so
    # every F-sized GEMM dimension runs on 224-row tiles that fill the chip (models/ffn.layer_fwd_t / layer_bwd_t)
    tp_transposed: bool = True
    # weight-gradient GEMM layout: "tn" (dW = dyᵀ·a, daᵀ·x: both operands through transposed LDS reads), "nn"
    # (transposed copies xᵀ / dyᵀ [D, T] from the producing epilogues; models/ffn.NNWgrad), "nn_w1" (dW1 only: xᵀ
    # copies; dW2 stays TN) or "nn_w2t" (nn with W2 stored as W2ᵀ [F, D]: both weight gradients written through the
    # transposed map); "auto" = nn_w2t where the engine supports it (GPU, bf16, 256x256 8-phase shapes without split-K,
    # no TP / SP / recompute, fused SGD / AdamW on split masters or stored gradients; DDP / ZeRO / FSDP meshes included)
    wgrad_layout: str = "auto"
    # W2's storage in the row-major layer: "auto" (transposed W2ᵀ [F, D] with the nn_w2t weight-gradient mode and on
    # row-major TP layers on the GPU, where it turns the dgrad into an NT GEMM),
    # "rowmajor", or "transposed" (any weight-gradient layout and mesh but the grouped weight-gradient pair; on the GPU bf16
    # with dW2 on unsplit 256x256 tiles and split masters under a fused optimizer; checkpoints stay logical [D, F])
    w2_storage: str = "auto"
    wgrad_stream: bool = False       # single device, fused optimizer: weight-gradient GEMMs on a second
                                     # stream, concurrent with the dgrad chain (CUs shared; epilogues overlap)
    wgrad_stream_max_tpc: float = 4.0  # wgrad_stream only while a weight gradient has <= this many 256x256 tiles
                                     # per CU (larger ones run serially: concurrent big GEMMs only split L2 / MALL)
    gemm_min_bpc: int = 0            # persistent GEMM grids: minimum blocks per CU (0 = auto: 2 when collectives
                                     # overlap the GEMMs, else 1)
    gemm_tiles_per_block: int = 0    # persistent GEMM blocks (process-wide): cap on tiles per block; 0 = auto
                                     # (8 -- the launcher picks the makespan-optimal count under it)
    fused_optimizer: bool = True     # fuse SGD/Adam into the wgrad GEMM epilogue when no grad collective
    side_optimizer: int = 0          # >0 (no grad collective, SGD): wgrad GEMMs store grads and a side stream
                                     # applies SGD on this many workgroups, overlapped with the next GEMMs;
                                     # <0: the same with the whole chip, any optimizer, split masters
    force_comm: bool = False         # run the DDP/FSDP collective path even at dp=1 (single-GPU RCCL check)
    fsdp_alias: bool = True          # FSDP at dp = 1: gathers / gradient writes alias the full buffers (size-1
                                     # collectives move nothing); False: the dp > 1 rings + real copying collectives
    zero_alias: bool = True          # ZeRO-2 at dp = 1: the reduce-scatter output is the gradient buffer itself and
                                     # the all-gather runs in place (size-1 collectives move nothing); False: a
                                     # separate gradient shard and an all-gather into a sink buffer -- real copying
                                     # RCCL collectives, the N > 1 schedule's per-GPU HBM traffic (bench zero_copy)
    force_tp_comm: bool = False      # with force_comm: also run the TP/SP collectives (forward output all-reduce
                                     # in chunks, deferred last-layer all-reduce, dx all-reduce / SP reduce-scatter
                                     # and all-gathers) over the size-1 tp communicator (single-GPU RCCL check)
    comm_backend: str = "torch"      # torch (ProcessGroupNCCL/gloo) | native (csrc/comm.cpp RCCL layer)
    tp_allreduce: str = "rccl"       # TP activation all-reduce: rccl (role communicator) | custom (csrc/car.hip) |
                                     # auto (time both on the [T, D] message at engine build, keep the faster)
    debug_sync: bool = False         # race screen: wait every collective at issue + device sync per layer
    master: str = "split"            # fp32 master weights of a bf16 run: split (the bf16 working copy + an int16
                                     # residual plane, together exactly the fp32 master: 4 B/param of weight state,
                                     # ops/master.py) | fp32 (a separate fp32 master next to the bf16 copy: 6 B/param)
    fp32_gemm: str = "bf16x6"        # fp32 compute GEMMs (process-wide): bf16x6 (exact 3-way bf16 split on the
                                     # bf16 MFMA kernels, fp32 accuracy) | mfma_f32 (fp32 MFMA kernel)

    @property
    def tokens(self) -> int:
        return self.batch_size * self.seq_len

    @property
    def torch_dtype(self) -> torch.dtype:
        return {"fp32": torch.float32, "bf16": torch.bfloat16}[self.dtype]

    @property
    def torch_grad_dtype(self) -> torch.dtype:
        return {"fp32": torch.float32, "bf16": torch.bfloat16}[self.grad_dtype]


def add_reference_args(p: argparse.ArgumentParser) -> None:
    p.add_argument("-s", "--num_steps", type=int, default=1)
    p.add_argument("-bs", "--batch_size", type=int, default=8)
    p.add_argument("-n", "--seq_len", type=int, default=1024)
    p.add_argument("-l", "--layers", type=int, default=1)
    p.add_argument("-d", "--model_size", type=int, default=4)
    p.add_argument("-m", "--method", type=int, default=0,
                   help="0=all, 1=1gpu, 2=DDP, 3=FSDP, 4=TP (MP), 5=hybrid FSDP/DDP x TP, "
                        "6=ZeRO-2 data parallel (sharded optimizer)")
    p.add_argument("-r", "--random_seed", type=int, default=0)


def add_extended_args(p: argparse.ArgumentParser) -> None:
    p.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32")
    p.add_argument("--grad_dtype", choices=["fp32", "bf16"], default=None)
    p.add_argument("--act", choices=["relu", "silu", "gelu"], default="relu")
    p.add_argument("--ffn_dim", type=int, default=0)
    p.add_argument("--gated", action="store_true")
    p.add_argument("--optimizer", choices=["sgd", "adam"], default="sgd")
    p.add_argument("--lr", type=float, default=LR)
    p.add_argument("--weight_decay", type=float, default=0.0)
    p.add_argument("--backend", choices=["auto", "nccl", "rccl", "gloo"], default="auto")
    p.add_argument("--comm", choices=["torch", "native"], default="torch",
                   help="communicator implementation for the role groups (native = C++ RCCL layer)")
    p.add_argument("--tp_allreduce", choices=["rccl", "custom", "auto"], default="rccl",
                   help="TP activation all-reduce: RCCL or the custom two-shot xGMI peer all-reduce")
    p.add_argument("--wgrad_layout", choices=["auto", "tn", "nn", "nn_w1", "nn_w2t"], default="auto",
                   help="weight-gradient GEMM layout (nn: transposed xᵀ / dyᵀ copies from the producing epilogues)")
    p.add_argument("--w2_storage", choices=["auto", "rowmajor", "transposed"], default="auto",
                   help="W2 stored row-major [D, F] or as W2ᵀ [F, D] (auto: with nn_w2t and on row-major TP layers)")
    p.add_argument("--nprocs", type=int, default=0, help="ranks to spawn (0 = all visible GPUs)")
    p.add_argument("--dp", type=int, default=0)
    p.add_argument("--tp", type=int, default=0)
    p.add_argument("--hybrid_dp_mode", choices=["ddp", "zero", "fsdp"], default="fsdp")
    p.add_argument("--sequence_parallel", action="store_true")
    p.add_argument("--recompute", choices=["none", "full"], default="none")
    p.add_argument("--bucket_mb", type=float, default=0.0)
    p.add_argument("--data", choices=["device", "cpu_compat"], default="cpu_compat")
    p.add_argument("--ckpt_dir", default="")
    p.add_argument("--ckpt_format", choices=["consolidated", "sharded"], default="consolidated")
    p.add_argument("--resume", default="")
    p.add_argument("--profile", default="", help="write a torch.profiler chrome trace (rank 0) to this path")
    p.add_argument("--metrics_jsonl", default="")
    p.add_argument("--strict", action="store_true", help="exit non-zero when method results disagree")
    p.add_argument("--master_port", type=int, default=29500)
    p.add_argument("--fp32_gemm", choices=["bf16x6", "mfma_f32"], default="bf16x6",
                   help="how --dtype fp32 GEMMs run: exact bf16 3-way split on the bf16 matrix cores, or fp32 MFMA")
    p.add_argument("--master", choices=["split", "fp32"], default="split",
                   help="fp32 master weights of a bf16 run: split (bf16 working copy + int16 residual, bit-exact, "
                        "4 B/param) or a separate fp32 buffer")
    p.add_argument("--debug_sync", action="store_true",
                   help="race screen: serialize every collective (must match the overlapped run bitwise)")
