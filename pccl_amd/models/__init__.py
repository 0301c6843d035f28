"""Reference workloads: MNIST MLP (end-to-end tests) and nanoGPT / GPT-2 124M (DDP and DiLoCo examples)."""
from .mlp import MLP
from .nanogpt import GPT, MI355X_BF16_DENSE_FLOPS, GPTConfig

__all__ = ["GPT", "GPTConfig", "MLP", "MI355X_BF16_DENSE_FLOPS"]
