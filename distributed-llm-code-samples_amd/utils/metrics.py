"""Throughput / FLOP accounting and step timing (the reference only prints one wall time per method,
train_ffns.py:378-382)."""
from __future__ import annotations

import json
import time

import torch

from .config import TrainConfig

# dense peaks used for MFU (MI355X_MICROARCH.md: bf16 MFMA ≈2.5 PF dense, fp32 MFMA 157.3 TF)
PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3}


def peak_tflops(dtype: str, fp32_gemm: str = "bf16x6") -> float:
    """The ceiling the step's GEMMs run against: fp32 on the bf16x6 split path executes six bf16 MFMA products
    per fp32 multiply-add, so its ceiling is the bf16 peak / 6 (417 TF), not the fp32 MFMA peak."""
    if dtype == "fp32" and fp32_gemm == "bf16x6":
        return PEAK_TFLOPS["bf16"] / 6
    return PEAK_TFLOPS.get(dtype, PEAK_TFLOPS["fp32"])


def flops_per_step(cfg: TrainConfig, tp: int = 1, recompute: str = "none", skip_dx0: bool = True) -> int:
    """Executed FLOPs per rank per step.

    Unit = one ``2·T·D·(F/tp)`` GEMM.  Per layer: forward 2 units (gated 3: x·W13ᵀ is 2F wide),
    backward 4 (gated 6): dW2, da, dx, dW1; ``recompute='full'`` adds the h recompute (1, gated 2) —
    the reference's 7 units per layer.  Layer 0 skips dx when ``skip_dx0``.
    """
    m = cfg.model
    unit = 2 * cfg.tokens * m.D * (m.F // tp)
    if m.gated:
        fwd, bwd, rec, dx = 3 * unit, 6 * unit, 2 * unit, 2 * unit
    else:
        fwd, bwd, rec, dx = 2 * unit, 4 * unit, unit, unit
    total = m.layers * (fwd + bwd + (rec if recompute == "full" else 0))
    if skip_dx0:
        total -= dx
    return int(total)


def model_flops_per_token(cfg: TrainConfig) -> int:
    """6·P model FLOPs per token (no recompute, all input grads)."""
    return 6 * cfg.model.num_params()


class StepTimer:
    """Per-step wall times with device synchronisation (first step reported separately as warm-up)."""

    def __init__(self, device: torch.device):
        self.device = device
        self.times: list[float] = []
        self._t0 = 0.0

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def start(self):
        self._sync()
        self._t0 = time.perf_counter()

    def stop(self):
        self._sync()
        self.times.append(time.perf_counter() - self._t0)

    def finish(self):
        pass

    @property
    def step_ms(self) -> list[float]:
        return [t * 1e3 for t in self.times]

    @property
    def steady_ms(self) -> float | None:
        ts = self.times[1:] if len(self.times) > 1 else self.times
        return (sum(ts) / len(ts) * 1e3) if ts else None


def mfu(tflops: float, dtype: str, fp32_gemm: str = "bf16x6") -> float:
    return tflops / peak_tflops(dtype, fp32_gemm)


def jsonl(path: str, rec: dict) -> None:
    if not path:
        return
    with open(path, "a") as f:
        f.write(json.dumps(rec) + "\n")
