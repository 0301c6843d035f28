"""MNIST MLP used by the DDP / DiLoCo end-to-end tests (reference python/tests/end_to_end/mnist_ddp/mnist_peer.py:52-82)."""
from __future__ import annotations

from typing import Sequence

import torch
import torch.nn as nn


class MLP(nn.Module):
    def __init__(self, input_size: int = 28 * 28, hidden_sizes: Sequence[int] = (128,), num_classes: int = 10):
        super().__init__()
        self.input_size = input_size
        dims = [input_size, *hidden_sizes]
        self.fc1 = nn.Linear(dims[0], dims[1])
        self.fcs = nn.ModuleList(nn.Linear(dims[i], dims[i + 1]) for i in range(1, len(dims) - 1))
        self.fc2 = nn.Linear(dims[-1], num_classes)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = torch.relu(self.fc1(x.reshape(-1, self.input_size)))
        for fc in self.fcs:
            x = torch.relu(fc(x))
        return self.fc2(x)
