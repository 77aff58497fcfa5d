"""MI355X-native distributed FFN training (DDP / FSDP / TP-MP / hybrid) — gfx950 HIP kernels + RCCL.

A from-scratch re-design of martin-kukla/distributed-llm-code-samples (``train_ffns.py``) for AMD
Instinct MI355X: explicit forward/backward of Transformer FFN stacks on hand-written CDNA4 MFMA GEMMs
with fused epilogues, fused optimizers, device-side mock data, and data / fully-sharded / tensor
parallelism over RCCL (xGMI) with one communicator + stream per communication role.

Importable as ``dllm`` (see ``dllm.py`` at the repository root).
"""
__version__ = "0.1.0"

import os as _os

# One HIP stream per communication role + compute + optimizer side streams: with HIP's default of 4 hardware
# queues per process, streams share queues round-robin and a collective enqueued on a stream that shares the
# compute stream's queue runs BETWEEN two GEMMs instead of under them (measured: every ZeRO-2 reduce-scatter copy
# of the N=1 forced-communicator step serialised with the next GEMM, profiles/r3/zero_hwqueue_*).  Give every
# stream its own queue.  Read when the HIP runtime initialises, so it must be set before the first HIP call --
# importing this package does that for bench.py, train_ffns.py, spawned ranks and torchrun ranks; an explicit
# GPU_MAX_HW_QUEUES in the environment wins.
_os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")

from .utils.config import ModelConfig, TrainConfig  # noqa: F401
