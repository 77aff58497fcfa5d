"""MI355X-native distributed FFN training (DDP / FSDP / TP-MP / hybrid) — gfx950 HIP kernels + RCCL.

A from-scratch re-design of martin-kukla/distributed-llm-code-samples (``train_ffns.py``) for AMD
Instinct MI355X: explicit forward/backward of Transformer FFN stacks on hand-written CDNA4 MFMA GEMMs
with fused epilogues, fused optimizers, device-side mock data, and data / fully-sharded / tensor
parallelism over RCCL (xGMI) with one communicator + stream per communication role.

Importable as ``dllm`` (see ``dllm.py`` at the repository root).
"""
__version__ = "0.1.0"

# Hardware queues: the package does not touch GPU_MAX_HW_QUEUES (HIP's default is 4 per process).  The compute
# stream's queue is kept free of other streams by utils/streams.reserve_compute_queue (bench.py / the launcher call it
# at process start); bench.py --hw_queues sets the variable explicitly for a run.

from .utils.config import ModelConfig, TrainConfig  # noqa: F401
