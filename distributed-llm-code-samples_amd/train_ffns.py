"""``train_ffns`` command line: the reference entry point (train_ffns.py:342-391), MI355X-native.

    python train_ffns.py --num_steps 16 --batch_size 8 --seq_len 1024 --layers 1 --model_size 8192 --method M

``M``: 0 = all methods, 1 = single GPU, 2 = DDP, 3 = FSDP (ZeRO-3 + DP), 4 = TP ("MP", Megatron),
5 = hybrid (FSDP / ZeRO / DDP) × TP, 6 = ZeRO-2 data parallel (reduce-scatter, sharded optimizer,
all-gather).  Reference flags keep their names and defaults; the extended flags
(``--dtype bf16 --act silu --gated --optimizer adam --ffn_dim …``) add the north-star features.

Stdout keeps the reference's lines (``ARGS:`` block, ``PARAMS:``, initial/final ``[:5,:5]`` slices,
``"<fn> takes <s> seconds"``, ``SoftAssertionError`` on a DDP/FSDP mismatch) and adds steady-state
tokens/s and TFLOP/s per method.  Unlike the reference it runs on exactly one GPU too (:25-27), checks
worker exit codes, also compares TP against 1-GPU, and ``--strict`` turns mismatches into exit code 1.
"""
from __future__ import annotations

import argparse
import os
import random
import sys
import time

import torch

from .parallel.launch import build_params, spawn
from .utils.config import METHODS, ModelConfig, TrainConfig, add_extended_args, add_reference_args
from .utils.metrics import jsonl, peak_tflops

FN_NAMES = {1: "train_1gpu", 2: "train_ddp", 3: "train_fsdp", 4: "train_tp", 5: "train_hybrid", 6: "train_zero"}


def make_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    add_reference_args(p)
    add_extended_args(p)
    p.add_argument("--init", choices=["auto", "cpu_compat", "device"], default="auto")
    return p


def config_from_args(a) -> TrainConfig:
    m = ModelConfig(model_size=a.model_size, ffn_dim=a.ffn_dim, layers=a.layers, act=a.act, gated=a.gated)
    return TrainConfig(model=m, batch_size=a.batch_size, seq_len=a.seq_len, num_steps=a.num_steps,
                       random_seed=a.random_seed, dtype=a.dtype, grad_dtype=a.grad_dtype or a.dtype,
                       optimizer=a.optimizer, lr=a.lr, weight_decay=a.weight_decay,
                       sequence_parallel=a.sequence_parallel, recompute=a.recompute, bucket_mb=a.bucket_mb,
                       data=a.data, comm_backend=a.comm, debug_sync=a.debug_sync, tp_allreduce=a.tp_allreduce, wgrad_layout=a.wgrad_layout,
                       w2_storage=a.w2_storage,
                       fp32_gemm=a.fp32_gemm, master=a.master)


def _fmt(t: torch.Tensor) -> str:
    return str(t)


def main(argv=None) -> int:
    a = make_parser().parse_args(argv)
    cfg = config_from_args(a)
    m = cfg.model
    print(f"ARGS:\n num_steps: {a.num_steps}\n BS: {a.batch_size}\n N: {a.seq_len}\n D: {m.D}\n FFN: {m.F}\n")
    seed = a.random_seed
    if seed == 0:
        seed = random.randint(1, 2**31 - 1)
        print(f"(random_seed 0: unseeded run, drew seed {seed})")

    backend = a.backend
    if backend in ("auto",):
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "rccl":
        backend = "nccl"
    n = a.nprocs or (torch.cuda.device_count() if backend == "nccl" else 2)
    init = a.init
    if init == "auto":
        init = "cpu_compat" if m.num_params() <= 2**27 else "device"

    num_params = m.num_params()
    print(f"PARAMS: {num_params:_} (size {4 * num_params / 1024 ** 3} GB)")
    print("\n")
    dev0 = torch.device("cuda", 0) if backend == "nccl" else torch.device("cpu")
    p0 = build_params(TrainConfig(model=ModelConfig(m.D, m.F, 1, m.act, m.gated), num_steps=cfg.num_steps), init,
                      seed, dev0)[0]
    print("initial layers_params[0]", p0["w1"].shape, p0["w2"].shape)
    print("initial layers_params[0]", _fmt(p0["w1"][:5, :5]), _fmt(p0["w2"][:5, :5]))
    del p0

    methods = [1, 2, 3, 4] if a.method == 0 else [a.method]
    opts_base = {"seed": seed, "init": init, "ckpt_dir": a.ckpt_dir, "ckpt_format": a.ckpt_format,
                 "resume": a.resume, "profile": a.profile, "return_params": True,
                 "return_full": a.method == 0 and num_params <= 2**26,
                 "tp": a.tp or n, "hybrid_dp_mode": a.hybrid_dp_mode}
    results = {}
    rc = 0
    for meth in methods:
        ranks = 1 if meth == 1 else n
        if meth == 5 and ranks % opts_base["tp"]:
            raise SystemExit(f"--tp {opts_base['tp']} does not divide {ranks} ranks")
        opts = dict(opts_base)
        if a.ckpt_dir and len(methods) > 1:
            opts["ckpt_dir"] = os.path.join(a.ckpt_dir, METHODS[meth])
        t0 = time.time()
        rec = spawn(ranks, cfg, meth, backend, a.master_port + meth, opts)
        t1 = time.time()
        results[meth] = rec
        name = FN_NAMES[meth]
        print(f"\n{name} takes {t1 - t0} seconds")
        if rec.get("shapes"):
            w1s, w2s = rec["shapes"][0]
            print(f"final {name} layers_params[0]", torch.Size(w1s), torch.Size(w2s))
            s1, s2 = rec["slices"][0]
            print(f"final {name} layers_params[0]", _fmt(s1), _fmt(s2))
        toks = rec["tokens_per_step_global"] * rec["steps"]
        steady = rec.get("steady_ms")
        line = {"method": name, "ranks": ranks, "wall_s": t1 - t0, "tokens_per_s_wall": toks / (t1 - t0)}
        if steady:
            line["steady_step_ms"] = steady
            line["tokens_per_s_steady"] = rec["tokens_per_step_global"] / (steady / 1e3)
            line["tflops_per_rank"] = rec["flops_per_step_rank"] / (steady / 1e3) / 1e12
            line["mfu_dense"] = line["tflops_per_rank"] / peak_tflops(cfg.dtype, cfg.fp32_gemm)
        if rec.get("peak_hbm_gib"):
            line["peak_hbm_gib_rank0"] = rec["peak_hbm_gib"]
        print("METRICS", line)
        jsonl(a.metrics_jsonl, line)

    if a.method == 0:
        rc |= _compare(results, 2, 3, "ddp", "fsdp", exact=True)
        rc |= _compare(results, 4, 1, "tp", "1gpu", exact=False)
    return rc if a.strict else 0


def _compare(results, i, j, ni, nj, exact: bool) -> int:
    A, B = results.get(i), results.get(j)
    if not A or not B:
        return 0
    bad = 0
    if A.get("params") and B.get("params"):
        for l, (pa, pb) in enumerate(zip(A["params"], B["params"])):
            for k in pa:
                ok = torch.allclose(pa[k], pb[k]) if exact else torch.allclose(pa[k], pb[k], rtol=1e-4, atol=1e-6)
                if not ok:
                    print(f"SoftAssertionError: L {l} {ni}[{k}] {pa[k]} {nj}[{k}] {pb[k]}")
                    bad = 1
    else:
        for l, ((a1, a2), (b1, b2)) in enumerate(zip(A["slices"], B["slices"])):
            for k, x, y in (("w1", a1, b1), ("w2", a2, b2)):
                if not torch.allclose(x, y, rtol=1e-4, atol=1e-6):
                    print(f"SoftAssertionError: L {l} {ni}[{k}] {x} {nj}[{k}] {y}")
                    bad = 1
    return bad


if __name__ == "__main__":
    sys.exit(main())
