"""HIP-graph capture of a whole training step (the MI355X replacement for a tracing compiler).

``GraphedStep`` captures device mock-data generation + forward + backward + fused optimizer of the
single-device / TP-free path once, then replays it: one ``hipGraphLaunch`` per step instead of ~60 kernel
launches through Python.  The per-step data seed lives in device memory (``rng_normal_pair_(..., seed_dev=)``), so each
replay draws new data; everything else is static (preallocated flat buffers, fixed shapes).

Restrictions (checked): no gradient collectives (``eng.fused_opt`` path), SGD (AdamW's bias correction is a
per-step kernel argument) and no concurrent weight-gradient stream.
"""
from __future__ import annotations

import torch

from ..ops.elementwise import STREAM_DY, STREAM_X, rng_normal_pair_
from .config import DLOSS_DX_COEF


class GraphedStep:
    def __init__(self, eng, tokens: int, model_size: int, warmup: int = 2):
        if eng.device.type != "cuda":
            raise ValueError("graph capture needs a GPU engine")
        if not eng.fused_opt or eng.cfg.optimizer != "sgd" or eng.mesh.world > 1:
            raise ValueError("GraphedStep supports the single-device fused-SGD path only")
        if eng.wg_stream is not None:
            # the concurrent weight-gradient stream carries Python-side events across steps (da/dx buffer
            # reuse), which a replayed capture cannot re-record
            raise ValueError("GraphedStep does not support the concurrent weight-gradient stream (wgrad_stream)")
        self.eng = eng
        dev = eng.device
        self.seed = torch.zeros(1, dtype=torch.int64, device=dev)
        self.x = torch.empty((tokens, model_size), dtype=eng.cd, device=dev)
        self.dy = torch.empty((tokens, model_size), dtype=eng.cd, device=dev)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for i in range(warmup):
                self.seed.fill_(-(i + 1))
                self._body()
        torch.cuda.current_stream(dev).wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._body()

    def _body(self):
        rng_normal_pair_(self.x, self.dy, 0, STREAM_X, 1.0, STREAM_DY, DLOSS_DX_COEF, seed_dev=self.seed)
        self.eng.train_step(self.x, self.dy)

    def step(self, seed: int) -> None:
        self.seed.fill_(int(seed))
        self.graph.replay()
