"""Model families: Transformer FFN stacks (ReLU/SiLU/GELU, optional SwiGLU gate) + the reference oracle."""
from .ffn import init_ffn_layer, init_linear_layer, layer_bwd, layer_fwd  # noqa: F401
