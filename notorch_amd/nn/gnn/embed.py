"""``GraphEmbedding`` (reference ``notorch/nn/gnn/embed.py:11-36``): sum-mode EmbeddingBag of the
integer atom / bond type columns into ``node_feats`` V x h and ``edge_feats`` E x h.

It produces the float inputs of the hot path; it is not itself on it (its fusion into the initial
gather is SURVEY §8(f) row 2), so it stays a plain PyTorch module.
"""
from __future__ import annotations

import torch.nn as nn

from notorch_amd.data.synth import DEFAULT_NUM_ATOM_TYPES, DEFAULT_NUM_BOND_TYPES

DEFAULT_HIDDEN_DIM = 256  # notorch/conf.py


class GraphEmbedding(nn.Module):
    def __init__(
        self,
        num_node_types: int = DEFAULT_NUM_ATOM_TYPES,
        num_edge_types: int = DEFAULT_NUM_BOND_TYPES,
        hidden_dim: int = DEFAULT_HIDDEN_DIM,
    ):
        super().__init__()
        self.node = nn.EmbeddingBag(num_node_types, hidden_dim, mode="sum")
        self.edge = nn.EmbeddingBag(num_edge_types, hidden_dim, mode="sum")

    def forward(self, G):
        return G.update(node_feats=self.node(G.node_feats), edge_feats=self.edge(G.edge_feats))

    @property
    def num_node_types(self) -> int:
        return self.node.num_embeddings

    @property
    def num_edge_types(self) -> int:
        return self.edge.num_embeddings
