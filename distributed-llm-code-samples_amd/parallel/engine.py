"""Unified FFN training engine: single device, DDP, FSDP (ZeRO-3), TP (Megatron MP) and 2-D hybrids.

The reference has four separate workers (train_ffns.py:101-116 single, :156-193 DDP, :197-287 FSDP,
:290-338 TP).  Here one engine covers all of them as points of a ``dp × tp`` mesh:

    method        dp_mode  dp  tp
    1 gpu         none     1   1
    2 DDP         ddp      n   1
    3 FSDP        fsdp     n   1
    4 TP / "MP"   none     1   n
    5 hybrid      ddp|fsdp d   t      (FSDP×TP for the Llama-3-8B-dims config)

MI355X-first memory design (288 GB HBM per GPU):

* **Flat buffers in completion order.**  Every rank owns one flat fp32 master buffer (plus its bf16
  compute copy, its gradient buffer and optional Adam moments; a bf16 run stores the fp32 master split, as the
  compute copy plus an int16 residual plane, ``ops/master.py``) holding, for ``l = L-1 … 0``, the
  layer's ``W2`` then ``W1`` (= the order the backward finishes them).  Any contiguous range is
  therefore a valid gradient bucket that becomes ready all at once — DDP buckets are plain views,
  collectives are zero-copy, and the optimizer runs over ranges with one fused kernel.
* **DDP**: wgrad GEMMs write straight into the flat gradient buffer; each bucket's all-reduce is issued
  on the ``dp_ar`` communicator the moment its last gradient is written, overlapping the rest of the
  backward (reference: per-tensor all-reduce, :164-165).  After the backward each bucket is waited
  for (a stream wait, not a host block) and updated in place by the fused optimizer, so early buckets'
  updates overlap late buckets' communication.
* **FSDP**: each rank keeps a row-shard (dim 0, as :265-266) of every weight.  Forward gathers layer
  l+1 while computing l; backward reuses the last layer's gathered weights and gathers l-1 while
  computing l (:236-250) — into a preallocated 2-slot ring with ``all_gather_into_tensor`` (no
  ``zeros_like``, no ``cat``).  Gradients go into a 2-slot full-layer ring and are reduce-scattered
  **asynchronously on their own communicator** (``dp_rs``), overlapping the next layer's backward —
  the overlap the reference could not get from one process group (:14, :252).  A shard's optimizer
  step runs as soon as its reduce-scatter is waited for.
* **TP**: W1 column-parallel (dim-0 rows), W2 row-parallel (dim-1 columns) (:316-319); per layer one
  all-reduce of ``y`` in forward (:303) and one of ``dx`` in backward (:309), the latter overlapped
  with the dW1 GEMM; the layer-0 input-grad all-reduce of the reference is skipped (its result is
  never used).  Optional sequence parallelism keeps activations T-sharded (reduce-scatter /
  all-gather instead of all-reduce).
"""
from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass

import torch

from ..models.ffn import (NNWgrad, deinterleave_w13, interleave_w13, layer_bwd, layer_bwd_t, layer_fwd, layer_fwd_t,
                          needs_preact, recompute_fwd1, wgrad_w1, wgrad_w2)
from ..ops.elementwise import adam_split_step_, adam_step_, cast_, sgd_split_step_, sgd_step_
from ..ops.master import join_flat, part_flat
from ..utils import streams
from ..utils.config import TrainConfig
from . import comm
from .mesh import Mesh

ALIGN = 64  # elements; keeps every view 128/256-B aligned for the LDS-DMA GEMM operand loads
# NN weight-gradient layout: transpose the step's x / dy on the weight-gradient stream (1) or the compute stream (0)
_TRANSPOSE_ON_SIDE = os.environ.get("DLLM_NN_TRANSPOSE_SIDE", "1") != "0"


def _round_up(n: int, a: int) -> int:
    return (n + a - 1) // a * a


def _nullctx():
    from contextlib import nullcontext

    return nullcontext()


@dataclass
class Entry:
    layer: int
    name: str            # "w1" (W1 or interleaved W13) | "w2"
    shape: tuple         # owned shape (shard shape under FSDP)
    full_shape: tuple    # local (TP-level) shape
    offset: int = 0

    @property
    def numel(self) -> int:
        return self.shape[0] * self.shape[1]


class _Hooks:
    def __init__(self, eng: "FFNTrainer", layer: int):
        self.eng, self.layer = eng, layer
        self.tp_work = None

    def after_w2(self):
        self.eng._grad_ready(self.layer, "w2")

    def after_dx(self, dx):
        e = self.eng
        if e.tp_comm:
            if e.tp_car is not None:
                self.tp_work = e.tp_car.all_reduce_async(dx)
            else:
                self.tp_work = comm.all_reduce(dx, e.mesh.group("tp"), async_op=True)
            if not e.cfg.tp_overlap:
                self.tp_work.wait()
                self.tp_work = None

    def after_w1(self):
        self.eng._grad_ready(self.layer, "w1")
        if self.tp_work is not None:
            self.tp_work.wait()
            self.tp_work = None


def gpu_chunk_count(T: int, D: int, F_loc: int, R1: int, c: int) -> int:
    """Largest chunk count <= ``c`` (halving) whose per-chunk forward GEMMs, ``[T/c, R1]`` (K = D) and ``[T/c, D]``
    (K = F_loc), need no split-K on the 256x256 kernels, i.e. still fill the chip on their own."""
    from ..ops.gemm import choose_ksplit

    c = max(1, c)
    while c > 1 and (T % c or choose_ksplit(T // c, R1, D) > 1 or choose_ksplit(T // c, D, F_loc) > 1):
        c //= 2
    return c


def wgrad_nn_shape_problem(T: int, D: int, F_loc: int, R1: int) -> str:
    """Why the NN weight-gradient layout cannot run at these shapes ('' = it can).  Every GEMM of the layout must sit
    on the 256x256 8-phase tiles, unsplit: the two weight gradients (dW2 [D, F] and dW1ᵀ [D, R1], K = T) and the two
    GEMMs whose epilogues write the transposed copies -- fwd-2 (y = a·W2ᵀ: M = T, N = D, K = F) and dx (M = T, N = D,
    K = R1).  E.g. T = 4224 (33 x 128 rows) passes the weight-gradient checks but not the copies' (T % 256)."""
    from ..ops.gemm import choose_ksplit, nn_wgrad_supported

    if T % 64 or not all(nn_wgrad_supported(*s) for s in ((D, F_loc, T), (D, R1, T), (T, D, F_loc), (T, D, R1))):
        return f"shapes (D={D}, F={F_loc}, T={T}) off the 256x256 8-phase tiles"
    if choose_ksplit(D, F_loc, T) > 1 or choose_ksplit(R1, D, T) > 1 or choose_ksplit(T, D, F_loc) > 1 \
            or choose_ksplit(T, D, R1) > 1:
        # small tile grids: the TN weight gradients / the fwd-2 and dx stores run split-K, which the transposed outputs
        # and copies do not (a different summation order: results would stop matching the TN layout's)
        return f"small tile grids (T={T}, D={D}, F={F_loc}) take split-K"
    return ""


class FFNTrainer:
    def __init__(self, cfg: TrainConfig, mesh: Mesh, device: torch.device):
        self.cfg, self.mesh, self.device = cfg, mesh, torch.device(device)
        if self.device.type == "cuda":
            # before the engine's side streams exist: keep them off the compute stream's hardware queue (idempotent;
            # bench.py / the launcher / init_distributed reserve earlier, before torch's stream pool exists)
            from ..utils.streams import reserve_compute_queue

            reserve_compute_queue(self.device)
        m = cfg.model
        D, F, L = m.D, m.F, m.layers
        t, d = mesh.tp, mesh.dp
        if F % t:
            raise ValueError(f"FFN dim {F} not divisible by tp={t} (train_ffns.py:317 needs equal chunks)")
        self.D, self.F, self.L = D, F, L
        self.F_loc = F // t
        self.gated = m.gated
        self.act = m.act
        if self.gated and self.F_loc % 16:
            raise ValueError("gated FFN needs (F / tp) % 16 == 0")
        self.R1 = (2 if self.gated else 1) * self.F_loc
        multi = d > 1 or cfg.force_comm
        self.fsdp = cfg.dp_mode == "fsdp" and multi
        self.ddp = cfg.dp_mode == "ddp" and multi
        self.zero = cfg.dp_mode == "zero" and multi
        if d > 1 and cfg.dp_mode == "none":
            raise ValueError("dp > 1 needs dp_mode ddp, zero or fsdp")
        if self.fsdp and (self.R1 % d or D % d):
            raise ValueError(f"FSDP needs W1 rows ({self.R1}) and D ({D}) divisible by dp={d} (train_ffns.py:266)")
        self.cd, self.gd = cfg.torch_dtype, cfg.torch_grad_dtype
        # TP collectives: a real tp axis, or forced over the size-1 tp communicator (force_tp_comm, single-GPU
        # check of the TP path: the same collectives, streams and waits as tp > 1)
        self.tp_comm = t > 1 or (cfg.force_comm and cfg.force_tp_comm and mesh.group("tp") is not None)
        self.sp = cfg.sequence_parallel and self.tp_comm
        T = cfg.tokens
        if self.sp and T % t:
            raise ValueError("sequence parallelism needs tokens % tp == 0")
        self.T = T
        # transposed-activation layout (models/ffn.layer_fwd_t): F/tp = 224k where 224-row tiles fill the chip better
        # (MP at tp 8: 1792 = 8 x 224 vs 7 x 256), so the F-sized GEMM dimensions run as M on 224-row tiles;
        # activations [F, T], W2 stored as W2ᵀ [F, D]
        from ..ops.gemm import use_m224

        self.tmode = (cfg.tp_transposed and self.device.type == "cuda" and not self.gated and not self.fsdp
                      and not self.zero and not self.sp and cfg.recompute == "none" and self.cd == torch.bfloat16
                      and use_m224(self.F_loc, T) and use_m224(self.F_loc, D) and T % 256 == 0)
        self.step_count = 0
        dev = self.device
        if dev.type == "cuda":
            from ..ops.gemm import set_fp32_mode, set_min_blocks_per_cu, set_tiles_per_block

            # gated stacks too since round 3 (persistent GLU / DGLU epilogues): L32 SwiGLU 167.6 vs 168.8 ms
            # (profiles/r3/gated_llama_dims_tpb_wgs_r3.txt)
            set_tiles_per_block(cfg.gemm_tiles_per_block or 8)
            set_fp32_mode(cfg.fp32_gemm)
            # collectives overlapping the GEMMs on a multi-rank mesh: RCCL kernels take CU slots, so keep >= 2 blocks
            # per CU.  Forced size-1 communicators launch no collective kernel (in place, nothing to move) and run
            # with one: hybrid 172.2-172.4 vs 175.8-176.1 ms, zero 30.5-30.7 vs 30.9-31.0
            # (profiles/r4/min_bpc_forcecomm_r4.txt)
            set_min_blocks_per_cu(cfg.gemm_min_bpc or (2 if mesh.world > 1 else 1))

        if cfg.debug_sync:
            comm.set_serialize(True)
        # custom xGMI all-reduce for the TP activation exchange (opt-in; gradients stay on RCCL)
        self.tp_car = None
        self.tp_ar_choice = None
        if cfg.tp_allreduce not in ("rccl", "custom", "auto"):
            raise ValueError(f"tp_allreduce {cfg.tp_allreduce!r}: expected rccl | custom | auto")
        if cfg.tp_allreduce in ("custom", "auto") and t > 1 and self.device.type == "cuda" and not cfg.sequence_parallel:
            from .car import CustomAllReduce

            # zero-copy: the exchanged activations (layer outputs xs[1..L], input gradients dxb) live in the car's
            # arena, which every TP peer maps; GEMMs write partials there and the all-reduce runs in place
            es = torch.empty(0, dtype=cfg.torch_dtype).element_size()
            per = (cfg.tokens * D * es + 255) // 256 * 256
            self.tp_car = CustomAllReduce(mesh.tp_ranks, self.device, cap_bytes=4096, tag=f"tp{mesh.dp_rank}",
                                          arena_bytes=(L + 3) * per)
            if cfg.tp_allreduce == "auto":
                self.tp_ar_choice = self._choose_tp_allreduce(cfg.tokens, D)
                if self.tp_ar_choice["choice"] == "rccl":
                    self.tp_car.destroy()
                    self.tp_car = None
            if self.tp_car is not None:
                mesh.groups["tp_car"] = self.tp_car

        # ---- optimizer / weight-gradient modes (they decide the parameter layout below) ----------------
        # no gradient collective (single device / pure TP): the optimizer runs inside the wgrad GEMMs and
        # no flat gradient buffer exists at all
        no_coll = not (self.ddp or self.fsdp or self.zero)
        # side-stream optimizer: wgrad GEMMs store the gradient, a low-occupancy SGD kernel on its own
        # stream updates the weight while the next GEMMs run; the forward waits per weight
        # (SGD only: a side-stream AdamW on the split master was measured 63 % slower on config 5 and removed, round 5,
        # profiles/r5/adamw_fused_vs_side_r5.txt)
        # side_optimizer < 0: the weight gradients are stored and each weight's flat update (SGD / AdamW, split masters)
        # runs on the side stream with the whole chip, overlapping the next GEMMs -- the schedule FSDP at dp = 1 runs.
        # An option: it measured slower than the fused epilogues (config 5 AdamW 185.8-187.2 vs 181.4-182.0 ms, the
        # flagship 29.45 vs 28.2 ms; profiles/r5/side_opt_whole_chip_r5.txt)
        self.side_opt = no_coll and dev.type == "cuda" and (
            (cfg.side_optimizer > 0 and cfg.optimizer == "sgd") or cfg.side_optimizer < 0)
        # Split master (bf16 SGD): the fp32 master is the bf16 working copy (hi) plus an int16 residual plane (lo),
        # bitwise the same fp32 values (ops/master.py).  4 B/param of weight state instead of 6 B, and every update
        # (fused wgrad epilogue or flat kernel) reads 4 B and writes 4 B per parameter instead of 4 B + 6 B.
        self.split = (cfg.master == "split" and self.cd == torch.bfloat16
                      and not (self.side_opt and cfg.side_optimizer > 0))   # the capped SGD kernel: fp32 masters
        if cfg.master not in ("split", "fp32"):
            raise ValueError(f"unknown master format {cfg.master!r}")
        self.fused_opt = cfg.fused_optimizer and no_coll and not self.side_opt
        # grouped weight-gradient pair (small tile grids: the MP / TP8 shard's dW2 [D, F/8] and dW1 [F/8, D] would each
        # run split-K plus a reduction pass): both in one launch of whole tiles, after dx (models/ffn.layer_bwd).  It
        # replaces the weight-gradient stream there: two part-empty grids have no tail worth filling
        self.pair_wgrads = False
        if dev.type == "cuda" and not self.tmode:
            from ..ops.gemm import pair_supported

            self.pair_wgrads = pair_supported(((D, self.F_loc, T), (self.R1, D, T)), self.cd)
        # NN weight-gradient layout (models/ffn.NNWgrad; buffers below).  It runs the backward serially: with the
        # concurrent weight-gradient stream it measured 0.35-0.45 ms per step slower than serial (3 interleaved pairs,
        # profiles/r5/nn_wgrad_step_ab_r5.txt), serial NN 0.1-0.4 ms faster than the TN layout on the stream
        # (DLLM_NN_CONCURRENT=1 keeps the stream for A/B runs).  Modes: nn_w1 = dW1 only; nn = dW2 as well, W2 row-major
        # (dW2's master rows 32 KiB apart); nn_w2t (auto) = dW2 as well with W2 stored transposed (W2ᵀ [F, D], the
        # transposed-activation mode's storage): dW2 then writes through the transposed map, fwd-2 runs NN and the
        # dgrad NT.  Flagship, serial, 3 interleaved triplets: tn 29.33-29.53, nn_w1 29.09-29.30, nn_w2t 28.26-28.30 ms
        # (profiles/r5/nn_wgrad_step_ab_r5.txt)
        mode = "nn_w2t" if cfg.wgrad_layout == "auto" else cfg.wgrad_layout
        self.wgrad_nn = self._wgrad_nn_supported() and mode in ("nn", "nn_w1", "nn_w2t")   # dW1 as NN (out_t)
        self.wgrad_nn_w2 = self.wgrad_nn and mode in ("nn", "nn_w2t")                        # dW2 as NN too
        # W2 stored as W2ᵀ [F_loc, D] in the row-major layer (self.w2s): the nn_w2t mode, or forced by cfg.w2_storage
        # (any wgrad layout: the TN weight gradient then writes through the transposed map too; CPU tests of the
        # storage, e.g. ZeRO-sharded checkpoints).  self.w2t: W2ᵀ storage in either layer form (tmode stores it too)
        if cfg.w2_storage not in ("auto", "rowmajor", "transposed"):
            raise ValueError(f"unknown w2_storage {cfg.w2_storage!r}")
        # auto: W2ᵀ with the nn_w2t weight-gradient mode, and on row-major TP layers (round 6), where the NN layout does
        # not run (its transposed copies would be of partial sums) but W2ᵀ storage still turns the dgrad da = dy·W2 into
        # an NT GEMM (both operands K-contiguous): config 5's SwiGLU dgrad 859 -> 700 us (NN -> NT), fwd-2 NT -> NN,
        # dW2 through the TN kernels' transposed output map (profiles/r6/config5_hybrid_phases_r6.txt)
        self.w2s = not self.tmode and (cfg.w2_storage == "transposed" or (cfg.w2_storage == "auto" and (
            (self.wgrad_nn and mode == "nn_w2t") or self._w2t_for_tp_layers())))
        if self.w2s and self.pair_wgrads:
            raise ValueError("w2_storage transposed: not with grouped weight-gradient pairs (they keep W2 row-major)")
        if self.w2s and dev.type == "cuda":
            # dW2 is written through the transposed output map on the GPU (any weight-gradient layout): the kernels
            # that have one -- bf16 operands on unsplit 256x256 tiles, and a fused optimizer on split masters only
            # (the transposed epilogues are 'store', 'sgd_split', 'adam_split').  Checked here, not at the first backward
            from ..ops.gemm import choose_ksplit, nn_wgrad_supported

            bad = []
            if self.cd != torch.bfloat16:
                bad.append("bf16 compute")
            if self.fused_opt and not self.split:
                bad.append("split masters with a fused optimizer")
            if not nn_wgrad_supported(D, self.F_loc, T) or choose_ksplit(D, self.F_loc, T) > 1:
                bad.append(f"dW2 [{D}, {self.F_loc}] (K = {T}) on unsplit 256x256 tiles")
            if bad:
                raise ValueError("w2_storage transposed needs " + ", ".join(bad))
        self.w2t = self.tmode or self.w2s

        # ---- flat owned parameter layout (completion order) ------------------------------------
        full = {"w2": (self.F_loc, D) if self.w2t else (D, self.F_loc), "w1": (self.R1, D)}
        self.entries: list[Entry] = []
        off = 0
        # ZeRO shards every bucket evenly over dp ranks: keep every entry a multiple of dp*ALIGN
        self.align = ALIGN * d if self.zero else ALIGN
        # layer 0 without an input gradient finishes dW1 BEFORE dW2 (see layer_bwd): its W1 gradient is
        # reduced, updated and re-gathered while the last GEMM (dW2) still runs, and the next forward's
        # first GEMM needs W1 first -- the step-boundary bubble shrinks to W2's collective, which
        # overlaps that first GEMM
        self.swap0 = cfg.skip_input_grad
        for l in reversed(range(L)):
            for name in self.layer_order(l):
                fs = full[name]
                own = (fs[0] // d, fs[1]) if self.fsdp else fs
                e = Entry(l, name, own, fs, off)
                off += _round_up(e.numel, self.align)
                self.entries.append(e)
        self.total = off
        self.entry = {(e.layer, e.name): e for e in self.entries}
        self._entry_index = {(e.layer, e.name): i for i, e in enumerate(self.entries)}

        # ---- DDP / ZeRO buckets ------------------------------------------------------------------
        self.buckets = []  # (start, end, last_entry_index)
        if self.ddp or self.zero:
            esize = torch.empty(0, dtype=self.gd).element_size()
            cap = int(cfg.bucket_mb * 2**20 / esize) if cfg.bucket_mb > 0 else 0
            start = 0
            for i, e in enumerate(self.entries):
                end = e.offset + _round_up(e.numel, self.align)
                if cap == 0 or end - start >= cap or i == len(self.entries) - 1:
                    self.buckets.append((start, end, i))
                    start = end
        if self.zero:
            # rank r owns [s + r*(e-s)/d, s + (r+1)*(e-s)/d) of every bucket; the owned pieces of all buckets
            # are stored back to back (shard offset goff): the fp32 master, the Adam moments and the reduced
            # gradient exist ONLY for the owned 1/dp (ZeRO-2), the compute copy stays full (it is what the
            # forward and backward read, refreshed by the per-bucket all-gather)
            self.bucket_shard = []
            goff = 0
            for s_, e_, _ in self.buckets:
                n = (e_ - s_) // d
                self.bucket_shard.append((s_ + mesh.dp_rank * n, s_ + (mesh.dp_rank + 1) * n, goff))
                goff += n
            self.shard_total = goff
        # ---- flat state ----------------------------------------------------------------------------
        # no gradient collective (single device / pure TP): the optimizer runs inside the wgrad GEMMs and
        # no flat gradient buffer exists at all
        nmaster = self.shard_total if self.zero else self.total
        self._master = None if self.split else torch.zeros(nmaster, dtype=torch.float32, device=dev)
        self.master_lo = torch.zeros(nmaster, dtype=torch.int16, device=dev) if self.split else None
        self._master_stage = None  # split: the fp32 master last materialised by `master` (written back by refresh_copy)
        self.shared_copy = self.cd == torch.float32 and not self.zero
        self.copy = self._master if self.shared_copy else torch.zeros(self.total, dtype=self.cd, device=dev)
        self.grads = torch.zeros(0 if self.fused_opt else self.total, dtype=self.gd, device=dev)
        if self.side_opt:
            self.opt_stream_side = self._side_stream("side_opt")
            self.opt_done = {}
        if cfg.optimizer == "adam":
            self.adam_m = torch.zeros(nmaster, dtype=torch.float32, device=dev)
            self.adam_v = torch.zeros(nmaster, dtype=torch.float32, device=dev)

        # ---- FSDP rings --------------------------------------------------------------------------
        if self.fsdp:
            # dp = 1 (forced communicators on one device): a rank's shard IS the full weight, so the gathers read and
            # write the working copy in place and the gradient GEMMs write the shard gradient directly -- size-1
            # collectives that move nothing (RCCL launches no kernel), the degenerate case of the N-rank schedule
            # (every wait, event and stream edge is still issued).  dp > 1: 2-slot gather / gradient rings.
            self.fsdp_alias = d == 1 and cfg.fsdp_alias
            self.wring = [{n: torch.empty(0 if self.fsdp_alias else full[n], dtype=self.cd, device=dev)
                           for n in ("w2", "w1")} for _ in range(2)]
            self.gring = [{n: torch.empty(0 if self.fsdp_alias else full[n], dtype=self.gd, device=dev)
                           for n in ("w2", "w1")} for _ in range(2)]
            self.ag_work = [None, None]     # per slot: {name: work} of the in-flight gather (None: landed)
            self.ag_layer = [-1, -1]
            self.rs_pending = [None, None]  # per slot: (layer, {name: work}) -- one reduce-scatter per weight
            self.ag_next = set()            # layers whose post-update gather for the next forward is in flight
            self.fsdp_stream = self._side_stream("fsdp")
            self.fsdp_tail_ev = None
            self.fsdp_upd = {}              # layer -> event: its shard update on the side stream (backward)

        # ---- activations -------------------------------------------------------------------------
        Tl = T // t if self.sp else T  # tokens held per rank between layers
        self.Tl = Tl
        car_arena = self.tp_car is not None and self.tp_car.arena is not None
        self.xs = [None] + [self.tp_car.arena_view((Tl, D), self.cd) if car_arena else
                            torch.empty((Tl, D), dtype=self.cd, device=dev) for _ in range(L)]
        keep = cfg.recompute == "none"
        nA = L if keep else 1
        ash = (self.F_loc, T) if self.tmode else (T, self.F_loc)      # transposed mode: [F, T]
        self.acts_a = [torch.empty(ash, dtype=self.cd, device=dev) for _ in range(nA)]
        self.need_h = needs_preact(self.act, self.gated)
        hsh = (self.R1, T) if self.tmode else (T, self.R1)
        self.acts_h = ([torch.empty(hsh, dtype=self.cd, device=dev) for _ in range(nA)]
                       if self.need_h else None)
        self.da = torch.empty(hsh, dtype=self.cd, device=dev)
        # ReLU: 1-bit activation-gradient masks (written by the forward's first GEMM, read by the dgrad)
        self.masks = None
        if cfg.relu_mask and self.act == "relu" and not self.gated and dev.type == "cuda":
            from ..ops.gemm import relu_mask_bytes, relu_mask_supported

            mM, mN = (self.F_loc, T) if self.tmode else (T, self.F_loc)
            if relu_mask_supported(mM, mN, D, self.cd):
                self.masks = [torch.empty(relu_mask_bytes(mM, mN), dtype=torch.uint8, device=dev)
                              for _ in range(nA)]
        # TP forward row chunks (see TrainConfig.tp_chunks): whole 256-row tiles per chunk; the ReLU bitmask is
        # written per chunk (tile-native layout, tile rows contiguous), so chunk GEMMs must stay on its kernels
        # On the GPU a chunk's two GEMMs must still fill the chip without split-K (fp32 partials + a reduction
        # pass per chunk cost more than the overlap buys), and a one-layer TP stack is not chunked at all: its
        # only output exchange is the last layer's, which overlaps the backward anyway (see train_step).
        self.tp_chunks = 1
        c = max(1, cfg.tp_chunks)
        if dev.type == "cuda":
            c = gpu_chunk_count(T, D, self.F_loc, self.R1, c)
        if self.tp_comm and not self.sp and not self.tmode and c > 1 and T % (256 * c) == 0 and L > 1:
            if self.masks is None:
                self.tp_chunks = c
            else:
                from ..ops.gemm import relu_mask_supported

                if relu_mask_supported(T // c, self.F_loc, D, self.cd):
                    self.tp_chunks = c
        # Sequence-parallel forward chunks: chunk i gathers every rank's i-th sub-slice of its T/tp rows, so the
        # gathered [T, *] buffers (inputs, activations, dy, partial outputs) hold the full T in a chunk-major row
        # order -- the same order in the forward, the backward and the ReLU masks; rows are independent in the FFN
        # and each rank's own T/tp rows keep their order.  The gathers of chunks i+1.. and the reduce-scatter of
        # chunk i run under chunk i's (i+1's) GEMMs.
        self.sp_chunks = 1
        if self.sp and c > 1 and T % (256 * c) == 0 and Tl % c == 0:
            if self.masks is None:
                self.sp_chunks = c
            else:
                from ..ops.gemm import relu_mask_supported

                if relu_mask_supported(T // c, self.F_loc, D, self.cd):
                    self.sp_chunks = c
        self._tp_pending = None
        self.before_backward = None  # optional callable at the start of every backward (data pipelines)
        # concurrent weight-gradient stream (single device, fused optimizer, kept activations): the dgrad
        # chain (da, dx) stays on the compute stream, dW2 / dW1 run on a side stream after the dgrad that
        # last reads the weight they update; da / dx buffers rotate so the side stream's reads never race
        # the next layers' writes
        # Only for weight gradients of at most `wgrad_stream_max_tpc` 256x256 tiles per CU: there the two streams'
        # GEMMs fill each other's last tile wave (flagship D4096: 4 per CU, 0.4-1.1 % faster); with many tiles per CU
        # nothing is left to fill and the two concurrent GEMMs only split L2 / MALL (D8192 F32768, 16 per CU: 131.5 vs
        # 117.8 ms serial; profiles/r3/wgrad_stream_tiles_per_cu_r3.txt)
        # grouped weight-gradient pair (small tile grids: the MP / TP8 shard's dW2 [D, F/8] and dW1 [F/8, D] would each
        # run split-K plus a reduction pass): both in one launch of whole tiles, after dx (models/ffn.layer_bwd).  It
        # replaces the weight-gradient stream there: two part-empty grids have no tail worth filling
        # (self.pair_wgrads and the NN weight-gradient mode are decided before the parameter layout, above)
        self.wg_stream = None
        wg_tiles = -(-self.R1 // 256) * -(-D // 256)
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count if dev.type == "cuda" else 256
        if (cfg.wgrad_stream and self.fused_opt and dev.type == "cuda" and not self.tp_comm and not self.sp
                and cfg.recompute == "none" and wg_tiles <= cfg.wgrad_stream_max_tpc * ncu and not self.pair_wgrads
                and not self.tmode and (not self.wgrad_nn or os.environ.get("DLLM_NN_CONCURRENT", "0") == "1")):
            self.wg_stream = self._side_stream("wgrad")
            self.da_ring = [self.da, torch.empty_like(self.da)]
            self.da_free = [None, None]
            self.dx_free = [None, None, None]
        self.dxb = [self.tp_car.arena_view((T, D), self.cd) if car_arena else
                    torch.empty((T, D), dtype=self.cd, device=dev)
                    for _ in range(3 if self.wg_stream is not None else 2)]
        if self.sp:
            self.xfull = torch.empty((T, D), dtype=self.cd, device=dev)       # gathered layer input
            self.yfull = torch.empty((T, D), dtype=self.cd, device=dev)       # partial output
            self.xs_full = [torch.empty((T, D), dtype=self.cd, device=dev) for _ in range(L)] if keep else None
            self.dyfull = torch.empty((T, D), dtype=self.cd, device=dev)
            self.dxs = [torch.empty((Tl, D), dtype=self.cd, device=dev) for _ in range(2)]
        # NN weight-gradient layout (models/ffn.NNWgrad): transposed copies xᵀ of every layer input (the previous layer's
        # fwd-2 epilogue writes them; layer 0's is transposed at the step start) and dyᵀ of every layer's output
        # gradient (the layer above's dx epilogue, rotating with dxb; the top layer's is transposed at the step start)
        self.xT = self.dxTb = self.dyT_top = None
        if self.wgrad_nn:
            self.xT = [torch.empty((D, T), dtype=self.cd, device=dev) for _ in range(L)]
        if self.wgrad_nn_w2:
            self.dxTb = [torch.empty((D, T), dtype=self.cd, device=dev) for _ in range(len(self.dxb))]
            self.dyT_top = torch.empty((D, T), dtype=self.cd, device=dev)

        # ---- DDP / ZeRO bucket state ----------------------------------------------------------------
        if self.ddp or self.zero:
            self.bucket_work = [None] * len(self.buckets)
            self.weight_buckets = {(l, n): sorted(b for b, (s_, e_, _) in enumerate(self.buckets)
                                                  if s_ < self.entry[(l, n)].offset + self.entry[(l, n)].numel
                                                  and self.entry[(l, n)].offset < e_)
                                   for l in range(L) for n in ("w1", "w2")}
            # the step-boundary buckets' optimizer (+ ZeRO all-gather) run on a side stream so the next
            # step's first GEMM does not queue behind the last collective; the forward waits per weight
            self.opt_stream = self._side_stream("opt")
            self.ddp_done = [None] * len(self.buckets)
        if self.zero:
            # dp = 1: the owned shard of every bucket is the whole bucket, so the reduced gradient IS the gradient
            # buffer (in-place size-1 reduce-scatter, no copy)
            # cfg.zero_alias False (bench.py zero_copy): a separate shard and an all-gather sink, so the size-1 RCCL
            # reduce-scatter / all-gather copy their bytes as the N > 1 collectives do
            self.zero_alias = d == 1 and cfg.zero_alias
            self.gshard = (self.grads[:self.shard_total] if self.zero_alias else
                           torch.zeros(self.shard_total, dtype=self.gd, device=dev))
            self.ag_sink = (torch.empty(self.total, dtype=self.cd, device=dev) if d == 1 and not self.zero_alias
                            else None)
            self.ag_pending = [None] * len(self.buckets)
            self.rs_issued_at = [None] * len(self.buckets)
        self._next_bucket = 0

    def input_transposes(self) -> tuple[torch.Tensor | None, torch.Tensor | None]:
        """The buffers a step's ``x`` / ``dy`` are transposed into (NN weight-gradient layout: layer 0's xᵀ, the top
        layer's dyᵀ; None where not used), for ``DeviceMockData.bind_transposed``."""
        if not self.wgrad_nn or self.sp:
            return None, None
        return self.xT[0], (self.dyT_top if self.wgrad_nn_w2 else None)

    def _w2t_for_tp_layers(self) -> bool:
        """``w2_storage='auto'`` on row-major TP layers: W2 stored as W2ᵀ when the GPU kernels that then run exist -- bf16,
        dW2 [D, F/tp] on unsplit 256x256 tiles (the TN transposed output map), split masters under a fused optimizer,
        no grouped weight-gradient pair."""
        if not (self.tp_comm and self.device.type == "cuda" and self.cd == torch.bfloat16 and not self.pair_wgrads):
            return False
        if self.fused_opt and not self.split:
            return False
        from ..ops.gemm import choose_ksplit, nn_wgrad_supported

        return nn_wgrad_supported(self.D, self.F_loc, self.T) and choose_ksplit(self.D, self.F_loc, self.T) == 1

    def _wgrad_nn_supported(self) -> bool:
        """Whether the weight gradients run in the NN layout (``cfg.wgrad_layout``; models/ffn.NNWgrad): GPU, bf16, the
        plain row-major layer (no TP / SP / transposed-activation mode / recompute / grouped pair / TP chunks),
        256x256 8-phase shapes, and a fused optimizer only on split masters (SGD / AdamW; stored gradients: any)."""
        cfg = self.cfg
        if cfg.wgrad_layout not in ("auto", "tn", "nn", "nn_w1", "nn_w2t"):
            raise ValueError(f"unknown wgrad_layout {cfg.wgrad_layout!r}")
        if cfg.wgrad_layout == "tn":
            return False
        from ..ops.gemm import _VARIANT, BF16_VARIANTS

        T, D = self.T, self.D
        why = []
        if self.device.type != "cuda" or self.cd != torch.bfloat16:
            why.append("GPU bf16 only")
        if self.tp_comm or self.sp or self.tmode or self.pair_wgrads:
            why.append("row-major data-parallel / single-device layers only")
        if cfg.recompute != "none":
            why.append("kept activations only")
        if self.fused_opt and not self.split:
            why.append("fused optimizer: split masters only")
        shape_why = wgrad_nn_shape_problem(T, D, self.F_loc, self.R1)
        if shape_why:
            why.append(shape_why)
        if BF16_VARIANTS.get(_VARIANT["name"], 0) not in (0, 3):
            why.append(f"GEMM variant {_VARIANT['name']}: transposed outputs run on the 8-phase staggered kernels only")
        if why and cfg.wgrad_layout in ("nn", "nn_w1", "nn_w2t"):
            raise ValueError(f"wgrad_layout {cfg.wgrad_layout}: " + "; ".join(why))
        return not why

    # ------------------------------------------------------------------------------------------------
    # views
    # ------------------------------------------------------------------------------------------------
    def _view(self, flat: torch.Tensor, e: Entry) -> torch.Tensor:
        return flat[e.offset:e.offset + e.numel].view(e.shape)

    def logical_view(self, flat: torch.Tensor, e: Entry) -> torch.Tensor:
        """The stored 2-D tensor of ``e`` in the logical [out, in] orientation (a transposed view of W2ᵀ in the
        transposed-activation layout; checkpoints read and write through it)."""
        v = self._view(flat, e)
        return v.t() if (self.w2t and e.name == "w2") else v

    @property
    def master(self) -> torch.Tensor:
        """The fp32 master state this rank stores (full layout, FSDP row shards, or the ZeRO owned-shard layout).

        fp32 format: the live buffer.  Split format: a new fp32 tensor joined from the bf16 working copy and the int16
        residual plane (read-only view of the state; writes go through ``flat_buffers`` + ``refresh_copy``)."""
        return self._master if not self.split else self._join_master()

    @property
    def master_numel(self) -> int:
        """Elements of this rank's fp32 master state (without joining a split master)."""
        return (self.master_lo if self.split else self._master).numel()

    @property
    def master_bytes(self) -> int:
        """Bytes of master-weight state besides the working copy: the fp32 master, or the split format's residual
        plane."""
        t = self.master_lo if self.split else self._master
        return t.numel() * t.element_size()

    def _hi_shard(self) -> list:
        """Split format: the working-copy ranges that hold this rank's master state, as (copy_lo, copy_hi, state_off)."""
        if self.zero:
            return [(ss, se, go) for ss, se, go in self.bucket_shard]
        return [(0, self.total, 0)]

    def master_slice(self, a: int, b: int) -> torch.Tensor:
        """fp32 master state [a, b) of this rank's master layout (split: joined for that range only)."""
        if not self.split:
            return self._master[a:b]
        out = torch.empty(b - a, dtype=torch.float32, device=self.device)
        for ca, cb, go in self._hi_shard():
            lo_, hi_ = max(a, go), min(b, go + (cb - ca))
            if lo_ < hi_:
                join_flat(self.copy[ca + lo_ - go:ca + hi_ - go], self.master_lo[lo_:hi_], out[lo_ - a:hi_ - a])
        return out

    def _join_master(self) -> torch.Tensor:
        out = torch.empty(self.master_lo.numel(), dtype=torch.float32, device=self.device)
        for a, b, go in self._hi_shard():
            join_flat(self.copy[a:b], self.master_lo[go:go + (b - a)], out[go:go + (b - a)])
        return out

    def _store_master(self, w: torch.Tensor) -> None:
        """Split format: set the master state from an fp32 buffer of the master layout (hi into the working copy's
        owned ranges, lo into the residual plane)."""
        for a, b, go in self._hi_shard():
            part_flat(w[go:go + (b - a)], self.copy[a:b], self.master_lo[go:go + (b - a)])

    def master_view(self, l: int, name: str) -> torch.Tensor:
        if self.zero:
            raise RuntimeError("ZeRO keeps only this rank's shard of the fp32 master (see full_flat)")
        if self.split:
            raise RuntimeError("split master: the fp32 master is copy_view + the residual plane (master_lo)")
        return self._view(self._master, self.entry[(l, name)])

    def _owned_segments(self, lo: int, hi: int):
        """ZeRO: the parts of flat range [lo, hi) this rank owns, as (flat_lo, flat_hi, shard_offset)."""
        for ss, se, go in self.bucket_shard:
            a, b = max(lo, ss), min(hi, se)
            if a < b:
                yield a, b, go + (a - ss)

    @torch.no_grad()
    def full_flat(self, shard: torch.Tensor) -> torch.Tensor:
        """ZeRO: all-gather a shard-layout fp32 buffer (master / Adam moment) into a new full-layout flat
        buffer (collective over dp; a transient -- nothing full-size is kept).  Other modes: returned as is."""
        if not self.zero:
            return shard
        full = torch.zeros(self.total, dtype=shard.dtype, device=shard.device)
        grp = self.mesh.group("dp_ag")
        for b, (s_, e_, _) in enumerate(self.buckets):
            ss, se, go = self.bucket_shard[b]
            comm.all_gather_into(full[s_:e_], shard[go:go + (se - ss)].clone(), grp, async_op=False)
        return full

    def copy_view(self, l: int, name: str) -> torch.Tensor:
        return self._view(self.copy, self.entry[(l, name)])

    def grad_view(self, l: int, name: str) -> torch.Tensor:
        return self._view(self.grads, self.entry[(l, name)])

    def _layer_bwd_concurrent(self, l, g, w1, w2, a, h, kw1, kw2, need_dx, gT=None):
        """One layer's backward with the weight-gradient GEMMs on ``wg_stream`` (same math and order per
        stream as ``layer_bwd``).  Edges: dW2 after da (da reads the W2 copy dW2's fused update rewrites),
        dW1 after dx (same for W1); buffers are reused only after the side stream's last read of them.
        ``gT`` (NN weight-gradient layout): gᵀ [D, T]; dx's epilogue then also writes dxᵀ into ``dxTb[j]``, which
        rotates (and is released) with ``dxb[j]``.  Returns (the next layer's g, its gᵀ or None)."""
        from ..ops.gemm import gemm

        nn = None
        main, side = torch.cuda.current_stream(self.device), self.wg_stream
        act = self.act
        da = self.da_ring[l % 2]
        if self.da_free[l % 2] is not None:
            main.wait_event(self.da_free[l % 2])
        if self.gated:   # [dg|du] interleaved [T, 2F] (as layer_bwd)
            gemm(g, w2, "nt" if self.w2s else "nn", out=da, epi="dglu", act=act, aux=h)
        else:
            gemm(g, w2, "nt" if self.w2s else "nn", out=da, epi="dact", act=act, aux=h if h is not None else a,
                 mask=self._mask(l))
        e_da = torch.cuda.Event()
        e_da.record(main)
        side.wait_event(e_da)
        j = l % 3
        if self.wgrad_nn:
            nn = NNWgrad(self.xT[l], gT, self.dxTb[j] if need_dx and self.wgrad_nn_w2 else None)
        if need_dx:
            with torch.cuda.stream(side):
                wgrad_w2(g, a, kw2, nn, self.w2s)                         # dW2 = dyᵀ·a
                e_dy = torch.cuda.Event()
                e_dy.record(side)
            if self.dx_free[j] is not None:
                main.wait_event(self.dx_free[j])
            dx = gemm(da, w1, "nn", out=self.dxb[j], aux_t=nn.dx_t if nn is not None else None)   # dx = da·W1
            self.dx_free[(l + 1) % 3] = e_dy                              # g / gᵀ (= dx of layer l+1) read
            e_dx = torch.cuda.Event()
            e_dx.record(main)
            side.wait_event(e_dx)
        with torch.cuda.stream(side):
            wgrad_w1(da, self.xs[l], kw1, nn)                             # dW1 = daᵀ·x
            if not need_dx:
                wgrad_w2(g, a, kw2, nn, self.w2s)                         # layer 0: dW2 last
            e_w = torch.cuda.Event()
            e_w.record(side)
        self.da_free[l % 2] = e_w
        if need_dx:
            return dx, (nn.dx_t if nn is not None else None)
        return g, None

    def _mask(self, l: int) -> torch.Tensor | None:
        if self.masks is None:
            return None
        return self.masks[l if self.cfg.recompute == "none" else 0]

    def layer_order(self, l: int) -> tuple[str, str]:
        """Order in which layer l's weight gradients complete in the backward (= flat layout order)."""
        return ("w1", "w2") if (l == 0 and self.swap0) else ("w2", "w1")

    def _layer_range(self, l: int) -> tuple[int, int]:
        first, last = (self.entry[(l, n)] for n in self.layer_order(l))
        return first.offset, last.offset + _round_up(last.numel, self.align)

    # ------------------------------------------------------------------------------------------------
    # parameters in / out (logical layout: per layer w1 [F,D], w2 [D,F] (+ w3 [F,D] if gated))
    # ------------------------------------------------------------------------------------------------
    def _local_from_full(self, p: dict) -> dict:
        t, r = self.mesh.tp, self.mesh.tp_rank
        Fl = self.F_loc
        w1 = p["w1"][r * Fl:(r + 1) * Fl]
        if self.gated:
            w1 = interleave_w13(w1, p["w3"][r * Fl:(r + 1) * Fl])
        w2 = p["w2"][:, r * Fl:(r + 1) * Fl]
        if self.w2t:
            w2 = w2.t().contiguous()   # stored as W2ᵀ [F_loc, D]
        return {"w1": w1, "w2": w2}

    def flat_buffers(self) -> dict:
        """Named flat fp32 state buffers as this rank stores them (checkpointed): full layout, FSDP row
        shards, or the ZeRO owned-shard layout (``bucket_shard``)."""
        if self.zero:
            self.zero_sync_state()
        self.side_sync()
        self.ddp_sync()
        self.fsdp_sync()
        out = {"params": self.master}
        if self.split:
            # a checkpoint load writes the fp32 master into this buffer; refresh_copy() splits it back (train_step
            # drops it, so a stale one is never written over newer state)
            self._master_stage = out["params"]
        if self.cfg.optimizer == "adam":
            out["adam_m"], out["adam_v"] = self.adam_m, self.adam_v
        return out

    @torch.no_grad()
    def _choose_tp_allreduce(self, T: int, D: int, iters: int = 5, warm: int = 2) -> dict:
        """``tp_allreduce="auto"``: time RCCL (the tp role communicator) against the custom peer all-reduce
        (``csrc/car.hip``, zero-copy arena) on the TP message itself, ``[T, D]`` in the compute dtype, on the real tp
        group; the faster one carries the activation exchange.  Both timings are the max over the tp ranks, so every
        rank makes the same choice.  Bandwidths: algorithm = bytes / time, bus = 2(n-1)/n x algorithm (ring
        convention).  A few ms at 64 MiB on xGMI (budget: well under 0.5 s)."""
        n = self.mesh.tp
        x = self.tp_car.arena_view((T, D), self.cd)   # the arena's first range (released below: xs[1] reuses it)
        x.normal_()
        nbytes = x.numel() * x.element_size()
        grp = self.mesh.group("tp")
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

        def timed(fn):
            for _ in range(warm):
                fn()
            ev[0].record()
            for _ in range(iters):
                fn()
            ev[1].record()
            torch.cuda.synchronize(self.device)
            return ev[0].elapsed_time(ev[1]) / iters

        t_rccl = timed(lambda: comm.all_reduce(x, grp, async_op=False))
        t_car = timed(lambda: self.tp_car.all_reduce(x))
        self.tp_car.check()
        self.tp_car._arena_next = 0
        tt = torch.tensor([t_rccl, t_car], dtype=torch.float64, device=self.device)
        if grp is not None:
            import torch.distributed as dist

            if isinstance(grp, dist.ProcessGroup):
                dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=grp)
            else:   # native communicator: MAX over the tp ranks through the default group
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_rccl, t_car = float(tt[0]), float(tt[1])

        def bw(ms):
            alg = nbytes / (ms * 1e-3) / 1e9
            return {"ms": round(ms, 4), "algbw_GBps": round(alg, 1), "busbw_GBps": round(alg * 2 * (n - 1) / n, 1)}

        return {"choice": "custom" if t_car < t_rccl else "rccl", "bytes": nbytes, "ranks": n,
                "rccl": bw(t_rccl), "custom": bw(t_car)}

    def load_full_params(self, layers: list[dict], flat: torch.Tensor | None = None) -> None:
        """Set parameters (or another flat state buffer) from full logical tensors (identical on every
        rank; CPU or device)."""
        if len(layers) != self.L:
            raise ValueError("layer count mismatch")
        is_master = flat is None
        target = (None if self.split else self._master) if is_master else flat
        d, dr = self.mesh.dp, self.mesh.dp_rank
        for l, p in enumerate(layers):
            loc = self._local_from_full(p)
            for name in ("w2", "w1"):
                src = loc[name]
                e = self.entry[(l, name)]
                if self.zero:
                    srcf = src.to(device=self.device, dtype=torch.float32).reshape(-1)
                    if is_master and self.split:
                        # every rank writes the whole working copy (hi) in the owner's rounding, the owned lo pieces
                        hi = self.copy[e.offset:e.offset + e.numel]
                        lo = torch.empty(e.numel, dtype=torch.int16, device=self.device)
                        part_flat(srcf, hi, lo)
                        for a, b, go in self._owned_segments(e.offset, e.offset + e.numel):
                            self.master_lo[go:go + (b - a)].copy_(lo[a - e.offset:b - e.offset])
                        continue
                    for a, b, go in self._owned_segments(e.offset, e.offset + e.numel):
                        target[go:go + (b - a)].copy_(srcf[a - e.offset:b - e.offset])
                    if is_master:
                        self._view(self.copy, e).copy_(srcf.view(e.shape))  # RNE cast, as cast_
                    continue
                if self.fsdp:
                    rows = src.shape[0] // d
                    src = src[dr * rows:(dr + 1) * rows]
                if is_master and self.split:   # per weight: no full-size fp32 transient
                    part_flat(src.to(device=self.device, dtype=torch.float32).reshape(-1),
                              self.copy[e.offset:e.offset + e.numel], self.master_lo[e.offset:e.offset + e.numel])
                    continue
                self._view(target, e).copy_(src.to(torch.float32))
        if is_master and not self.split and not self.shared_copy and not self.zero:
            cast_(self._master, self.copy)
        if self.fsdp and is_master:
            self.fsdp_sync()
            self.ag_next.clear()  # gathered rings hold the old weights

    @torch.no_grad()
    def refresh_copy(self) -> None:
        """Recompute the compute-dtype working copy from the fp32 master after the master was written
        directly (checkpoint load).  ZeRO: every rank casts its shard and all-gathers (collective)."""
        if self.fsdp:
            self.fsdp_sync()
            self.ag_next.clear()  # gathered rings hold the old weights
        if self.split:
            # the fp32 master was written through the buffer flat_buffers() handed out (checkpoint load)
            if self._master_stage is not None:
                self._store_master(self._master_stage)
                self._master_stage = None
        elif self.shared_copy:
            return
        elif not self.zero:
            cast_(self._master, self.copy)
            return
        if not self.zero:
            return
        grp = self.mesh.group("dp_ag")
        for b, (s_, e_, _) in enumerate(self.buckets):
            ss, se, go = self.bucket_shard[b]
            if not self.split:
                self.copy[ss:se].copy_(self._master[go:go + (se - ss)])
            src = self.copy[ss:se].clone() if self.device.type != "cuda" else self.copy[ss:se]
            comm.all_gather_into(self.copy[s_:e_], src, grp, async_op=False)

    @torch.no_grad()
    def zero_sync_state(self) -> None:
        """ZeRO: make the current stream wait for every in-flight parameter all-gather (checkpoint, readout,
        teardown).  The fp32 state stays sharded; ``full_flat`` gathers a full copy when one is needed."""
        if not self.zero:
            return
        for b in range(len(self.buckets)):
            self._zero_wait_ag(b)

    @torch.no_grad()
    def local_params(self, flat: torch.Tensor | None = None) -> list[dict]:
        """This TP rank's full local (unsharded over dp) fp32 tensors of a flat buffer, w1 de-interleaved.
        Collective over the dp group under FSDP."""
        self.side_sync()
        self.ddp_sync()
        self.fsdp_sync()
        # split masters outside ZeRO: join each entry on its own (no full-size fp32 transient)
        per_entry = flat is None and self.split and not self.zero
        src = None if per_entry else (self.master if flat is None else flat)
        if self.zero:
            self.zero_sync_state()
            src = self.full_flat(src)
        out = []
        for l in range(self.L):
            p = {}
            for name in ("w1", "w2"):
                e = self.entry[(l, name)]
                mv = self.master_slice(e.offset, e.offset + e.numel).view(e.shape) if per_entry else self._view(src, e)
                if self.fsdp:   # row shards of the STORED matrix (W2ᵀ: rows are F)
                    full = torch.empty(self.entry[(l, name)].full_shape, dtype=torch.float32, device=self.device)
                    comm.all_gather_into(full, mv.contiguous(), self.mesh.group("dp_ag"), async_op=False)
                    mv = full
                if self.w2t and name == "w2":
                    mv = mv.t()   # logical [D, F_loc] from the stored W2ᵀ
                p[name] = mv
            if self.gated:
                w1, w3 = deinterleave_w13(p["w1"])
                p["w1"], p["w3"] = w1, w3
            out.append(p)
        return out

    @torch.no_grad()
    def gather_full_params(self, flat: torch.Tensor | None = None) -> list[dict] | None:
        """Full logical fp32 tensors on CPU at global rank 0 (None elsewhere).  Collective."""
        loc = self.local_params(flat)
        res = []
        for p in loc:
            q = {}
            for name, t in p.items():
                parts = comm.gather_to_rank0(t.contiguous(), self.mesh.group("tp"))
                q[name] = torch.cat(parts, dim=1 if name == "w2" else 0)
            res.append(q)
        return res if self.mesh.rank == 0 else None

    # ------------------------------------------------------------------------------------------------
    # optimizer over a flat range
    # ------------------------------------------------------------------------------------------------
    def _fused_wgrad_kw(self, l: int, name: str) -> dict:
        cfg = self.cfg
        if self.split:
            kw = {"out": self._view(self.master_lo, self.entry[(l, name)]), "epi": cfg.optimizer + "_split",
                  "lr": cfg.lr, "aux_out": self.copy_view(l, name)}
        else:
            kw = {"out": self.master_view(l, name), "epi": cfg.optimizer, "lr": cfg.lr}
            if not self.shared_copy:
                kw["aux_out"] = self.copy_view(l, name)
        if cfg.optimizer == "adam":
            e = self.entry[(l, name)]
            kw.update(betas=(cfg.adam_b1, cfg.adam_b2), eps=cfg.adam_eps, wd=cfg.weight_decay, step=self.step_count,
                      opt_m=self._view(self.adam_m, e), opt_v=self._view(self.adam_v, e))
        return kw

    def _opt(self, s: int, e: int) -> None:
        cfg = self.cfg
        if self.split:  # full or FSDP-shard layout: the residual plane shares the working copy's offsets
            if cfg.optimizer == "sgd":
                sgd_split_step_(self.master_lo[s:e], self.copy[s:e], self.grads[s:e], cfg.lr)
            else:
                adam_split_step_(self.master_lo[s:e], self.copy[s:e], self.grads[s:e], self.adam_m[s:e],
                                 self.adam_v[s:e], self.step_count, cfg.lr, cfg.adam_b1, cfg.adam_b2, cfg.adam_eps,
                                 cfg.weight_decay)
            return
        master, grad = self._master[s:e], self.grads[s:e]
        copy = None if self.shared_copy else self.copy[s:e]
        if cfg.optimizer == "sgd":
            sgd_step_(master, grad, cfg.lr, copy=copy)
        else:
            adam_step_(master, grad, self.adam_m[s:e], self.adam_v[s:e], self.step_count, cfg.lr,
                       cfg.adam_b1, cfg.adam_b2, cfg.adam_eps, cfg.weight_decay, copy=copy)

    # ------------------------------------------------------------------------------------------------
    # communication hooks
    # ------------------------------------------------------------------------------------------------
    def _grad_ready(self, l: int, name: str) -> None:
        if self.side_opt:
            e = self.entry[(l, name)]
            s_, e_ = e.offset, e.offset + e.numel
            st = self.opt_stream_side
            st.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(st):
                if self.cfg.side_optimizer < 0:
                    self._opt(s_, e_)             # whole chip, any optimizer, split or fp32 masters
                else:
                    copy = None if self.shared_copy else self.copy[s_:e_]
                    sgd_step_(self._master[s_:e_], self.grads[s_:e_], self.cfg.lr, copy=copy,
                              max_blocks=self.cfg.side_optimizer)
                ev = torch.cuda.Event()
                ev.record(st)
            self.opt_done[(l, name)] = ev
            return
        if self.zero:
            idx = self._entry_index[(l, name)]
            while self._next_bucket < len(self.buckets) and self.buckets[self._next_bucket][2] <= idx:
                b = self._next_bucket
                s_, e_, _ = self.buckets[b]
                ss, se, go = self.bucket_shard[b]
                self.bucket_work[b] = comm.reduce_scatter_into(self.gshard[go:go + (se - ss)], self.grads[s_:e_],
                                                               self.mesh.group("dp_rs"), async_op=True)
                self.rs_issued_at[b] = l
                self._next_bucket += 1
        elif self.ddp:
            idx = self._entry_index[(l, name)]
            while self._next_bucket < len(self.buckets) and self.buckets[self._next_bucket][2] <= idx:
                b = self._next_bucket
                s, e, _ = self.buckets[b]
                self.bucket_work[b] = comm.all_reduce(self.grads[s:e], self.mesh.group("dp_ar"), async_op=True)
                self._next_bucket += 1
        elif self.fsdp:
            # one reduce-scatter per weight, issued the moment its gradient GEMM is done: the first weight's
            # collective runs under the layer's remaining GEMMs instead of waiting for both
            slot = l % 2
            w = comm.reduce_scatter_into(self.grad_view(l, name), self._fsdp_gbuf(l, name), self.mesh.group("dp_rs"),
                                         async_op=True)
            if self.rs_pending[slot] is None or self.rs_pending[slot][0] != l:
                self.rs_pending[slot] = (l, {})
            self.rs_pending[slot][1][name] = w

    def _zero_finish(self, b: int, side: bool = False) -> None:
        """Bucket b's reduce-scatter is done -> update the owned shard -> all-gather the new bf16 copy.
        ``side``: do it on ``opt_stream`` instead of the compute stream."""
        if side and self.opt_stream is not None:
            self.opt_stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.opt_stream):
                self._zero_finish(b)
            return
        self.bucket_work[b].wait()
        self.bucket_work[b] = None
        s_, e_, _ = self.buckets[b]
        ss, se, go = self.bucket_shard[b]
        n = se - ss
        cfg = self.cfg
        g = self.gshard[go:go + n]
        bf16_copy = self.cd == torch.bfloat16
        copy = self.copy[ss:se] if bf16_copy else None  # bf16: written by the optimizer kernel itself
        master = None if self.split else self._master[go:go + n]
        if self.split and cfg.optimizer == "sgd":
            sgd_split_step_(self.master_lo[go:go + n], copy, g, cfg.lr)
        elif self.split:
            adam_split_step_(self.master_lo[go:go + n], copy, g, self.adam_m[go:go + n], self.adam_v[go:go + n],
                             self.step_count, cfg.lr, cfg.adam_b1, cfg.adam_b2, cfg.adam_eps, cfg.weight_decay)
        elif cfg.optimizer == "sgd":
            sgd_step_(master, g, cfg.lr, copy=copy)
        else:
            adam_step_(master, g, self.adam_m[go:go + n], self.adam_v[go:go + n], self.step_count, cfg.lr,
                       cfg.adam_b1, cfg.adam_b2, cfg.adam_eps, cfg.weight_decay, copy=copy)
        if not bf16_copy:
            self.copy[ss:se].copy_(master)  # fp32 compute: the working copy is a separate full buffer
        src = self.copy[ss:se]
        if self.device.type != "cuda":
            src = src.clone()  # gloo: keep input and output of the all-gather disjoint
        dst = self.copy[s_:e_] if self.ag_sink is None else self.ag_sink[s_:e_]   # sink: dp = 1, zero_alias off
        self.ag_pending[b] = comm.all_gather_into(dst, src, self.mesh.group("dp_ag"), async_op=True)
        self.rs_issued_at[b] = None

    def _ddp_wait(self, l: int, name: str) -> None:
        for b in self.weight_buckets[(l, name)]:
            ev = self.ddp_done[b]
            if ev is not None:
                torch.cuda.current_stream(self.device).wait_event(ev)
                self.ddp_done[b] = None

    def ddp_sync(self) -> None:
        if self.ddp:
            for (l, n) in list(self.weight_buckets):
                self._ddp_wait(l, n)

    def _side_wait(self, l: int, name: str) -> None:
        ev = self.opt_done.pop((l, name), None)
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)

    def side_sync(self) -> None:
        """Make the current stream wait for every pending side-stream update (checkpoint / readout)."""
        if self.side_opt:
            for k in list(self.opt_done):
                self._side_wait(*k)

    def _zero_wait_ag(self, b: int) -> None:
        if self.ag_pending[b] is not None:
            self.ag_pending[b].wait()
            self.ag_pending[b] = None

    def _fsdp_finish_rs(self, slot: int, names=None) -> None:
        """Wait for the slot's pending reduce-scatters (``names``: only those weights) and update their shards."""
        pend = self.rs_pending[slot]
        if pend is None:
            return
        l, works = pend
        for n in [n for n in self.layer_order(l) if n in works and (names is None or n in names)]:
            works.pop(n).wait()
            e = self.entry[(l, n)]
            self._opt(e.offset, e.offset + e.numel)
        if not works:
            self.rs_pending[slot] = None

    def _fsdp_finish_rs_side(self, slot: int) -> None:
        """Backward: the slot's previous layer (l + 2) -- wait for its reduce-scatters on the compute stream (its
        gradient ring slot is rewritten next) and update its shards on the side stream, off the compute stream's
        critical path.  The next forward's gather of that layer waits for the update (``fsdp_upd``)."""
        pend = self.rs_pending[slot]
        if pend is None:
            return
        st = self.fsdp_stream
        if st is None:
            self._fsdp_finish_rs(slot)
            return
        lay, works = pend
        # dp = 1: no gradient ring slot to protect, the side stream's own wait suffices (hybrid 171.7 / 172.2 vs
        # 172.4 / 172.7 ms with the wait, profiles/r4/fsdp_dp1_rs_wait_r4.txt)
        if not self.fsdp_alias:
            for w in works.values():
                w.wait()
        with torch.cuda.stream(st):
            self._fsdp_finish_rs(slot)
            ev = torch.cuda.Event()
            ev.record(st)
        self.fsdp_upd[lay] = ev

    def _fsdp_gather(self, l: int, names=("w2", "w1")) -> None:
        slot = l % 2
        grp = self.mesh.group("dp_ag")
        ev = self.fsdp_upd.pop(l, None)
        if ev is not None:  # the shard was updated on the side stream
            torch.cuda.current_stream(self.device).wait_event(ev)
        if self.ag_layer[slot] != l or self.ag_work[slot] is None:
            self.ag_work[slot] = {}
        # the weights' shard all-gathers as one group (native: one fused RCCL launch)
        w = comm.all_gather_into_many([(self._fsdp_wbuf(l, n), self.copy_view(l, n)) for n in names], grp,
                                      async_op=True)
        for n in names:
            self.ag_work[slot][n] = w
        self.ag_layer[slot] = l

    def _fsdp_weight(self, l: int, name: str) -> torch.Tensor:
        """Layer l's gathered weight ``name`` from the ring, after a (stream) wait for its gather."""
        slot = l % 2
        if self.ag_layer[slot] != l:
            raise RuntimeError(f"FSDP ring slot {slot} holds layer {self.ag_layer[slot]}, wanted {l}")
        works = self.ag_work[slot]
        if works is not None and works.get(name) is not None:
            works.pop(name).wait()
        return self._fsdp_wbuf(l, name)

    def _fsdp_wbuf(self, l: int, name: str) -> torch.Tensor:
        """Where layer l's gathered weight lives: its ring slot, or (dp = 1) the working copy itself."""
        return self.copy_view(l, name) if self.fsdp_alias else self.wring[l % 2][name]

    def _fsdp_gbuf(self, l: int, name: str) -> torch.Tensor:
        """Where layer l's full weight gradient is written: its ring slot, or (dp = 1) the shard gradient itself."""
        return self.grad_view(l, name) if self.fsdp_alias else self.gring[l % 2][name]

    def _fsdp_weights(self, l: int) -> tuple[torch.Tensor, torch.Tensor]:
        return self._fsdp_weight(l, "w1"), self._fsdp_weight(l, "w2")

    def _fsdp_tail(self) -> None:
        """Step boundary of FSDP: the last two layers' gradients (layers 1 and 0) are reduce-scattered, their
        shards updated and re-gathered for the next forward on a side stream, in the order the next forward needs
        them: layer 0's first-completed weight (W1 without a layer-0 input gradient: its chain runs under the
        dW2 GEMM), layer 1, then layer 0's other weight.  The forward then waits per weight (W1 before the first
        GEMM, W2 before the second), so only the last chain's tail is exposed (reference: synchronous
        reduce-scatter, gather at the start of the next forward, train_ffns.py:236-259, TODO :14/:252)."""
        L = self.L
        st = self.fsdp_stream
        first, second = self.layer_order(0)
        plan = [(0, (first,))] + ([(1, ("w2", "w1"))] if L >= 2 else []) + [(0, (second,))]
        ctx = torch.cuda.stream(st) if st is not None else _nullctx()
        with ctx:
            for l, names in plan:
                # the chain waits only for its reduce-scatters (ordered after the gradient GEMMs that wrote the
                # grad ring, and after every earlier GEMM reading this layer's ring slot), not for the compute
                # stream's later GEMMs
                self._fsdp_finish_rs(l % 2, names)
                self._fsdp_gather(l, names)
                self.ag_next.add(l)
            if st is not None:
                self.fsdp_tail_ev = torch.cuda.Event()
                self.fsdp_tail_ev.record(st)

    def fsdp_sync(self) -> None:
        """Make the current stream wait for the step-boundary updates / gathers (checkpoint, readout)."""
        if self.fsdp and self.fsdp_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.fsdp_stream)

    def _side_stream(self, role: str):
        """The engine's stream for side-work ``role`` (utils/streams.py picks its hardware queue); None off the GPU."""
        return streams.side_stream(self.device, role, owner=self) if self.device.type == "cuda" else None

    # ------------------------------------------------------------------------------------------------
    # one training step
    # ------------------------------------------------------------------------------------------------
    def train_step(self, x: torch.Tensor, dy: torch.Tensor) -> torch.Tensor:
        """Forward + backward + gradient communication + optimizer for one batch.

        ``x``/``dy`` are ``[T, D]`` in the compute dtype (under sequence parallelism, the full T: each
        rank keeps its T/tp slice).  Returns the forward output ``y`` (this rank's view).
        """
        cfg = self.cfg
        L, act, gated = self.L, self.act, self.gated
        self._master_stage = None   # a checkpoint buffer handed out before this step is stale from here on
        self.step_count += 1
        keep = cfg.recompute == "none"
        tpg = self.mesh.group("tp")
        if self.sp:
            t, r = self.mesh.tp, self.mesh.tp_rank
            x = x[r * self.Tl:(r + 1) * self.Tl]
            dy = dy[r * self.Tl:(r + 1) * self.Tl]
        self.xs[0] = x
        if self.wgrad_nn:
            # the NN weight-gradient layout's transposed copies of the step's inputs (every other layer's come out of
            # the producing GEMM epilogues): layer 0's xᵀ and the top layer's dyᵀ.  Only weight-gradient GEMMs read
            # them, so with a weight-gradient stream they are made there, off the forward's critical path (the stream
            # is joined at the end of every step, and x / dy are not rewritten before the next step)
            from ..ops.gemm import transpose_bf16

            # A batch from DeviceMockData.bind_transposed arrives with them already drawn (tag _dllm_t, consumed here)
            need_dy = self.wgrad_nn_w2 and getattr(dy, "_dllm_t", None) is not self.dyT_top
            need_x = getattr(x, "_dllm_t", None) is not self.xT[0]
            for t_ in (x, dy):
                if getattr(t_, "_dllm_t", None) is not None:
                    t_._dllm_t = None
            side = self.wg_stream if (self.wg_stream is not None and _TRANSPOSE_ON_SIDE) else None
            if side is not None and (need_x or need_dy):
                side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
                if need_dy:
                    transpose_bf16(dy, self.dyT_top)
                if need_x:
                    transpose_bf16(x, self.xT[0])

        # ---------------- forward ----------------
        mark = self._mark("forward")
        fsdp_w2 = None
        if self.fsdp and 0 not in self.ag_next:
            self._fsdp_gather(0)
        for l in range(L):
            if self.fsdp:
                w1 = self._fsdp_weight(l, "w1")   # W2 is waited for right before the second GEMM
                w2 = self._fsdp_wbuf(l, "w2")
                self.ag_next.discard(l)
                if l + 1 < L and (l + 1) not in self.ag_next:
                    self._fsdp_gather(l + 1)

                def fsdp_w2(l=l):
                    self._fsdp_weight(l, "w2")
            else:
                if self.zero:
                    for b in self.weight_buckets[(l, "w1")]:
                        self._zero_wait_ag(b)
                if self.side_opt:
                    self._side_wait(l, "w1")
                if self.ddp:
                    self._ddp_wait(l, "w1")
                w1, w2 = self.copy_view(l, "w1"), self.copy_view(l, "w2")
            a = self.acts_a[l if keep else 0]
            h = (self.acts_h[l if keep else 0]) if self.need_h else None
            if self.sp:
                if self.zero:
                    for b in self.weight_buckets[(l, "w2")]:
                        self._zero_wait_ag(b)
                if self.side_opt:
                    self._side_wait(l, "w2")
                if self.ddp:
                    self._ddp_wait(l, "w2")
                if fsdp_w2 is not None:
                    fsdp_w2()
                self._sp_fwd(l, self.xs_full[l] if keep else self.xfull, w1, w2, a, h)
            else:
                before2 = fsdp_w2
                if self.zero:
                    def before2(l=l):
                        for b in self.weight_buckets[(l, "w2")]:
                            self._zero_wait_ag(b)
                elif self.side_opt:
                    def before2(l=l):
                        self._side_wait(l, "w2")
                elif self.ddp:
                    def before2(l=l):
                        self._ddp_wait(l, "w2")
                if self.tp_chunks > 1:
                    self._tp_fwd_chunked(l, w1, w2, a, h, before2)
                    continue
                if self.tmode:
                    layer_fwd_t(self.xs[l], w1, w2, act, a, h, self.xs[l + 1], before_fwd2=before2, mask=self._mask(l))
                else:
                    layer_fwd(self.xs[l], w1, w2, act, gated, a, h, self.xs[l + 1], before_fwd2=before2,
                              mask=self._mask(l), y_t=self.xT[l + 1] if self.wgrad_nn and l + 1 < L else None,
                              w2t=self.w2s)
                if self.tp_comm:
                    last = l == L - 1
                    if self.tp_car is not None:
                        w = self.tp_car.all_reduce_async(self.xs[l + 1])
                    else:
                        # the next layer reads it at once: synchronous, on the compute stream (no stream hops)
                        w = comm.all_reduce(self.xs[l + 1], tpg, async_op=last)
                    if last:
                        self._tp_pending = [w]
                    else:
                        w.wait()
        # The last layer's TP output exchange (all-reduce / SP reduce-scatter of y) is left in flight: nothing in
        # the backward reads y (dL/dy is an input), so it runs under the backward GEMMs and is waited at the end
        # of the step (reference: synchronous all_reduce(y) before the backward, train_ffns.py:300-303).
        y_pending, self._tp_pending = self._tp_pending, None
        y = self.xs[L]

        self._unmark(mark)
        # ---------------- backward ----------------
        mark = self._mark("backward")
        if self.before_backward is not None:
            self.before_backward()  # e.g. the data pipeline starts drawing the next batch (utils/data.py)
        self._next_bucket = 0
        if self.fsdp and self.fsdp_tail_ev is not None:
            # the previous step's tail reduce-scatters read the gradient ring this backward rewrites
            torch.cuda.current_stream(self.device).wait_event(self.fsdp_tail_ev)
            self.fsdp_tail_ev = None
        if self.fsdp and L >= 2 and self.ag_layer[(L - 2) % 2] != L - 2:
            # the forward left layers L-1 and L-2 in the ring; weights do not change until the
            # optimizer runs, so the reference's re-gather of L-2 (:245) is skipped when still resident
            self._fsdp_gather(L - 2)
        g = dy
        gT = self.dyT_top if self.wgrad_nn_w2 else None    # gᵀ: the NN weight-gradient layout's dW2 operand
        for l in reversed(range(L)):
            if self.fsdp:
                if l < L - 1:
                    w1, w2 = self._fsdp_weights(l)
                    if l >= 1:
                        self._fsdp_gather(l - 1)
                else:
                    w1, w2 = self._fsdp_weights(l)
                slot = l % 2
                self._fsdp_finish_rs_side(slot)  # slot's previous grads (layer l+2) must be reduced first
                gw1, gw2 = self._fsdp_gbuf(l, "w1"), self._fsdp_gbuf(l, "w2")
            elif self.fused_opt:
                w1, w2 = self.copy_view(l, "w1"), self.copy_view(l, "w2")
                gw1, gw2 = self._fused_wgrad_kw(l, "w1"), self._fused_wgrad_kw(l, "w2")
            else:
                w1, w2 = self.copy_view(l, "w1"), self.copy_view(l, "w2")
                gw1, gw2 = self.grad_view(l, "w1"), self.grad_view(l, "w2")
            if keep:
                a = self.acts_a[l]
                h = self.acts_h[l] if self.need_h else None
            else:
                a = self.acts_a[0]
                h = self.acts_h[0] if self.need_h else None
            need_dx = l > 0 or not cfg.skip_input_grad
            hooks = _Hooks(self, l)
            if self.sp:
                # gather dy (T-sharded) and the layer input; dx partial -> reduce-scatter
                for w in self._sp_gather(self.dyfull, g):
                    w.wait()
                xin = self.xs_full[l] if keep else self.xfull
                if not keep:
                    for w in self._sp_gather(xin, self.xs[l]):
                        w.wait()
                    recompute_fwd1(xin, w1, act, gated, a, h, mask=self._mask(l))
                hooks_sp = _SPHooks(self, l)
                dxp = layer_bwd(self.dyfull, xin, w1, w2, act, gated, a, h, gw1, gw2, self.da,
                                self.dxb[l % 2] if need_dx else None, hooks_sp, mask=self._mask(l),
                                dx_first=cfg.tp_overlap, pair_wgrads=self.pair_wgrads, w2t=self.w2s)
                if dxp is not None:
                    for w in hooks_sp.rs_work or ():
                        w.wait()
                    g = self.dxs[l % 2]
            elif self.wg_stream is not None:
                g, gT = self._layer_bwd_concurrent(l, g, w1, w2, a, h, gw1, gw2, need_dx, gT)
            elif self.tmode:
                dx = layer_bwd_t(g, self.xs[l], w1, w2, act, a, h, gw1, gw2, self.da,
                                 self.dxb[l % 2] if need_dx else None, hooks, mask=self._mask(l))
                if dx is not None:
                    g = dx
            else:
                if not keep:
                    recompute_fwd1(self.xs[l], w1, act, gated, a, h, mask=self._mask(l))
                nn = (NNWgrad(self.xT[l], gT, self.dxTb[l % 2] if need_dx and self.wgrad_nn_w2 else None)
                      if self.wgrad_nn else None)
                dx = layer_bwd(g, self.xs[l], w1, w2, act, gated, a, h, gw1, gw2, self.da,
                               self.dxb[l % 2] if need_dx else None, hooks, mask=self._mask(l),
                               dx_first=self.tp_comm and cfg.tp_overlap, pair_wgrads=self.pair_wgrads, nn=nn,
                               w2t=self.w2s)
                if dx is not None:
                    g = dx
                    gT = nn.dx_t if nn is not None else None
            if self.zero:
                # reduce-scatters issued during an earlier layer have had a full layer of compute to
                # finish: update those shards now (1/dp of the optimizer work, off the tail), on the side stream
                # so the shard update and its all-gather overlap the next GEMMs instead of running between them
                for b, at in enumerate(self.rs_issued_at):
                    if at is not None and at > l:
                        self._zero_finish(b, side=True)

        if self.wg_stream is not None:
            # the next forward reads the updated weights (and reuses every activation buffer)
            torch.cuda.current_stream(self.device).wait_stream(self.wg_stream)
        self._unmark(mark)
        # ---------------- optimizer ----------------
        mark = self._mark("optimizer_tail")
        if self.zero:
            for b, at in enumerate(self.rs_issued_at):
                if at is not None:
                    self._zero_finish(b, side=True)
        elif self.ddp:
            # every bucket's update runs on the side stream behind its all-reduce (stream waits, no host block), in
            # the order the next forward needs the weights (layer 0's buckets first), so the later layers' updates
            # overlap the next forward's first GEMMs; the forward waits per weight
            for b in reversed(range(len(self.buckets))):
                s, e, _ = self.buckets[b]
                if self.opt_stream is not None:
                    self.opt_stream.wait_stream(torch.cuda.current_stream(self.device))
                    with torch.cuda.stream(self.opt_stream):
                        self.bucket_work[b].wait()
                        self._opt(s, e)
                        ev = torch.cuda.Event()
                        ev.record(self.opt_stream)
                    self.ddp_done[b] = ev
                else:
                    self.bucket_work[b].wait()
                    self._opt(s, e)
        elif self.fsdp:
            self._fsdp_tail()
        elif not self.fused_opt and not self.side_opt:
            self._opt(0, self.total)
        self._unmark(mark)
        for w in y_pending or ():
            w.wait()
        if cfg.debug_sync:
            self.check_health()
        return y

    def _sp_parts(self, full: torch.Tensor, local: torch.Tensor) -> list:
        """(chunk of the gathered [T, *] buffer, this rank's matching sub-slice of its T/tp rows) per SP chunk."""
        c = self.sp_chunks
        rf, rl = self.T // c, self.Tl // c
        return [(full[i * rf:(i + 1) * rf], local[i * rl:(i + 1) * rl]) for i in range(c)]

    def _sp_gather(self, full: torch.Tensor, local: torch.Tensor) -> list:
        """Async all-gather of every rank's T/tp rows into ``full`` in the chunk-major order (one per chunk)."""
        tpg = self.mesh.group("tp")
        return [comm.all_gather_into(f, lo, tpg, async_op=True) for f, lo in self._sp_parts(full, local)]

    def _sp_scatter(self, local: torch.Tensor, full: torch.Tensor) -> list:
        """Async reduce-scatter of a chunk-major partial ``full`` into this rank's T/tp rows (one per chunk)."""
        tpg = self.mesh.group("tp")
        return [comm.reduce_scatter_into(lo, f, tpg, async_op=True) for f, lo in self._sp_parts(full, local)]

    def _sp_fwd(self, l: int, xin: torch.Tensor, w1, w2, a, h) -> None:
        """Sequence-parallel forward of layer l in ``sp_chunks`` chunks: every chunk's input gather is issued up
        front (chunk i+1's runs under chunk i's GEMMs), chunk i's partial output is reduce-scattered as soon as
        its GEMMs are done (under chunk i+1's).  The next layer's gathers queue behind these reduce-scatters on
        the TP communicator; the last layer's are waited at the end of the forward.  (Reference TP: synchronous
        all_reduce of y, train_ffns.py:300-303.)"""
        c = self.sp_chunks
        rf = self.T // c
        mask = self._mask(l)
        mband = (rf // 256) * (self.F_loc // 256) * 8192 if mask is not None else 0  # mask bytes per chunk
        # the previous layer's reduce-scatters wrote xs[l]: on RCCL they precede these gathers on the TP stream
        # anyway (the waits are stream waits); gloo may run queued collectives concurrently
        for w in self._tp_pending or ():
            w.wait()
        gathers = self._sp_gather(xin, self.xs[l])
        tpg = self.mesh.group("tp")
        pend = []
        for i, (yf, yl) in enumerate(self._sp_parts(self.yfull, self.xs[l + 1])):
            gathers[i].wait()
            r = slice(i * rf, (i + 1) * rf)
            layer_fwd(xin[r], w1, w2, self.act, self.gated, a[r], h[r] if h is not None else None, yf,
                      mask=mask[i * mband:(i + 1) * mband] if mask is not None else None, w2t=self.w2s)
            pend.append(comm.reduce_scatter_into(yl, yf, tpg, async_op=True))
        self._tp_pending = pend

    def _tp_fwd_chunked(self, l: int, w1, w2, a, h, before2) -> None:
        """Tensor-parallel forward of layer l in ``tp_chunks`` row chunks: chunk i's partial-output all-reduce
        is issued as soon as its two GEMMs are done and runs while chunk i+1 computes; the next layer's chunk i
        waits (stream wait, no host block) only for that chunk's all-reduce.  Rows are independent in the FFN,
        so the results equal the one-all-reduce-per-layer schedule (reference: sync all_reduce(y),
        train_ffns.py:300-303)."""
        c, x, y = self.tp_chunks, self.xs[l], self.xs[l + 1]
        rows = self.T // c
        mask = self._mask(l)
        mband = (rows // 256) * (self.F_loc // 256) * 8192 if mask is not None else 0  # mask bytes per chunk
        prev, works = self._tp_pending, []
        for ci in range(c):
            r = slice(ci * rows, (ci + 1) * rows)
            if prev is not None:
                prev[ci].wait()
            layer_fwd(x[r], w1, w2, self.act, self.gated, a[r], h[r] if h is not None else None, y[r],
                      before_fwd2=before2 if ci == 0 else None,
                      mask=mask[ci * mband:(ci + 1) * mband] if mask is not None else None, w2t=self.w2s)
            if self.tp_car is not None:
                works.append(self.tp_car.all_reduce_async(y[r]))
            else:
                works.append(comm.all_reduce(y[r], self.mesh.group("tp"), async_op=True))
        self._tp_pending = works

    def check_health(self) -> None:
        """Raise if an asynchronous failure was recorded on the device: a timed-out barrier of the custom
        TP all-reduce (whose results are then NaN-poisoned, csrc/car.hip).  Synchronises the device; called
        after every step under ``debug_sync`` and by the drivers after their final synchronize."""
        if self.tp_car is not None:
            self.tp_car.check()

    # ------------------------------------------------------------------------------------------------
    # phase annotation: roctx ranges (DLLM_ROCTX=1, rocprofv3 --marker-trace) and optional HIP-event
    # phase timers (``enable_phase_timing``); both are no-ops otherwise
    # ------------------------------------------------------------------------------------------------
    def enable_phase_timing(self, on: bool = True) -> None:
        from ..utils.profiling import PhaseTimer

        self.phase_timer = PhaseTimer(on) if on else None

    def phase_summary(self) -> dict:
        pt = getattr(self, "phase_timer", None)
        return pt.summary() if pt is not None else {}

    def _mark(self, name: str):
        from ..utils.profiling import roctx_push

        roctx_push(name)
        pt = getattr(self, "phase_timer", None)
        if pt is None or not pt.enabled:
            return (name, None)
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return (name, ev)

    def _unmark(self, tok) -> None:
        from ..utils.profiling import roctx_pop

        roctx_pop()
        name, ev = tok
        if ev is not None:
            end = torch.cuda.Event(enable_timing=True)
            end.record()
            self.phase_timer.events.append((name, ev, end))


class _SPHooks(_Hooks):
    """Sequence-parallel variant: the partial dx is reduce-scattered over T (asynchronously, overlapping the
    weight-gradient GEMMs that follow it in the ``dx_first`` order); the caller waits after the layer."""

    rs_work = None

    def after_dx(self, dx):
        e = self.eng
        self.rs_work = e._sp_scatter(e.dxs[self.layer % 2], dx)
        if not e.cfg.tp_overlap:
            for w in self.rs_work:
                w.wait()
            self.rs_work = None

    def after_w1(self):
        self.eng._grad_ready(self.layer, "w1")
