"""Parallelism: process mesh + role communicators, the unified DDP/FSDP/TP engine, spawning."""
from .engine import FFNTrainer  # noqa: F401
from .mesh import Mesh, init_distributed  # noqa: F401
