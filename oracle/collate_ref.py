"""Pure-Python restatement of ``BatchedGraph.from_graphs`` (notorch/data/models/graph.py:186-223).
TEST INFRASTRUCTURE ONLY — see oracle/__init__.

Returns plain tensors: node_feats, edge_feats, edge_index, rev_index, batch_node_index,
batch_edge_index, size.  ``rev_offset="nodes"`` is the reference as written (line 200 offsets
rev_index by the running NODE count, line 204); ``"edges"`` is the corrected variant.
"""
from __future__ import annotations

import torch


def from_graphs(Gs, rev_offset: str = "nodes") -> dict:
    node_featss, edge_featss, edge_indices, rev_indices = [], [], [], []
    batch_node_indices, batch_edge_indices = [], []
    offset = 0
    eoffset = 0
    for i, G in enumerate(Gs):                                         # :196
        node_featss.append(G.node_feats)                               # :197
        edge_featss.append(G.edge_feats)                               # :198
        edge_indices.append(G.edge_index + offset)                     # :199
        rev_indices.append(G.rev_index + (offset if rev_offset == "nodes" else eoffset))  # :200
        batch_node_indices.extend([i] * len(G.node_feats))             # :201
        batch_edge_indices.extend([i] * len(G.edge_feats))             # :202
        offset += len(G.node_feats)                                    # :204
        eoffset += len(G.edge_feats)
    return dict(
        node_feats=torch.cat(node_featss, dim=0),                      # :206
        edge_feats=torch.cat(edge_featss, dim=0),                      # :207
        edge_index=torch.cat(edge_indices, dim=1).long(),              # :208
        rev_index=torch.cat(rev_indices, dim=0).long(),                # :209
        batch_node_index=torch.tensor(batch_node_indices, dtype=torch.long),  # :210
        batch_edge_index=torch.tensor(batch_edge_indices, dtype=torch.long),  # :211
        size=i + 1,                                                    # :212
    )
