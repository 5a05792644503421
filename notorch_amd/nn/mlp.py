"""``MLP`` head (reference ``notorch/nn/mlp.py:9-68``), SURVEY §8(f) row 4.

The head runs on the readout's B x h rows (4096 x 300 at config 2: ~0.7 GFLOP per 300 x 300 layer), a
plain dense GEMM that PyTorch-ROCm hands to hipBLASLt, so it is built from ``nn.Linear`` on purpose:
no hand-written kernel would beat the library at this shape, and it is off the timed path.  What the
drop-in needs is the same module tree: ``Linear, act, Dropout, Linear, ..., Linear`` (the dropout
before the first layer and the activation after the last one are left out), optionally followed by
``nn.Unflatten``, so the ``state_dict`` keys (``0.weight``, ``3.weight``, ...) and the output shape
match the reference's.
"""
from __future__ import annotations

from collections.abc import Sequence
from math import prod

import torch.nn as nn

DEFAULT_HIDDEN_DIM = 256  # notorch/conf.py:11


def MLP(
    input_dim: int,
    output_size: int | Sequence[int],
    hidden_dim: int = DEFAULT_HIDDEN_DIM,
    num_layers: int = 1,
    dropout: float = 0.0,
    activation: type[nn.Module] = nn.ReLU,
) -> nn.Sequential:
    """input_dim -> num_layers hidden layers of hidden_dim -> output_size (an int, or a shape the last
    dimension is unflattened into).  One activation and one dropout module, shared by every block,
    as in the reference (neither holds parameters)."""
    shape = None if isinstance(output_size, int) else tuple(output_size)
    out_dim = output_size if shape is None else prod(shape)
    act, drop = activation(), nn.Dropout(dropout)
    widths = [input_dim, *([hidden_dim] * num_layers), out_dim]
    mods: list[nn.Module] = []
    for k, (d_in, d_out) in enumerate(zip(widths[:-1], widths[1:])):
        if k > 0:  # between two linear layers: activation, then dropout
            mods += [act, drop]
        mods.append(nn.Linear(d_in, d_out))
    mlp = nn.Sequential(*mods)
    if shape is not None:
        mlp.append(nn.Unflatten(-1, shape))
    return mlp
