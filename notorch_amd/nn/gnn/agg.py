"""Graph readouts (reference ``notorch/nn/gnn/agg.py:15-47``) on the segment-reduce kernel.

``Sum`` / ``Mean`` / ``Max`` reduce ``G.node_feats`` over the nodes of each molecule
(``batch_node_index``, ``dim_size=len(G)``) with torch_scatter semantics: mean divides by
``max(count, 1)``, an empty molecule reads 0 for every reduction.  ``Min`` is added for
completeness of the ``Reduction`` domain (notorch/types.py:57).

``Gated`` and ``SDPAttention`` (agg.py:50-86) are SURVEY §8(f) row 4 — not provided yet.
"""
from __future__ import annotations

from abc import abstractmethod

import torch.nn as nn
from torch import Tensor

from notorch_amd.nn.gnn import _engine


class Aggregation(nn.Module):
    reduce: str = "sum"

    @abstractmethod
    def forward(self, G, **kwargs) -> Tensor:
        pass


class _SegmentReadout(Aggregation):
    def forward(self, G, **kwargs) -> Tensor:
        X = G.node_feats
        if X.device.type != "cuda":
            raise RuntimeError(
                f"notorch_amd.{type(self).__name__} runs on ROCm devices only; got '{X.device}'"
            )
        mol_ptr, mol_perm = _engine.mol_layout(G)
        return _engine.segment_reduce_readout(
            X.contiguous(), mol_ptr, mol_perm, len(G), self.reduce, G.batch_node_index
        )


class Sum(_SegmentReadout):
    """agg.py:23-29: ``scatter_sum(node_feats, batch_node_index, dim=0, dim_size=len(G))``."""

    reduce = "sum"


class Mean(_SegmentReadout):
    """agg.py:32-38: ``scatter_mean(...)``."""

    reduce = "mean"


class Max(_SegmentReadout):
    """agg.py:41-47: ``scatter_max(...)[0]``."""

    reduce = "max"


class Min(_SegmentReadout):
    reduce = "min"
