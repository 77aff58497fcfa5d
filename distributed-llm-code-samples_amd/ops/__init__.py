"""Device ops: MFMA GEMMs with fused FFN epilogues, RNG, fused optimizers (HIP on GPU, torch on CPU)."""
from .activations import act_fwd, act_grad  # noqa: F401
from .elementwise import adam_step_, cast_, rng_normal_, sgd_step_  # noqa: F401
from .gemm import gemm  # noqa: F401
