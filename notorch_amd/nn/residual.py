"""``Residual`` wrapper (reference ``notorch/nn/residual.py:21-28``).

``ChempropBlock`` never calls it on the device path: the residual add is fused into
``nt_dmpnn_update``.  It is kept so the module tree and ``state_dict`` keys
(``layers.{i}.module.update.0.weight``) are identical to the reference, and so a standalone
``Residual(ChempropLayer)`` still computes ``inputs[0] + module(*inputs)``.
"""
from __future__ import annotations

import torch.nn as nn


class Residual(nn.Module):
    def __init__(self, module: nn.Module):
        super().__init__()
        self.module = module

    def forward(self, *inputs):
        return inputs[0] + self.module(*inputs)
