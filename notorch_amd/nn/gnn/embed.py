"""``GraphEmbedding`` (reference ``notorch/nn/gnn/embed.py:11-36``): sum-mode EmbeddingBag of the
integer atom / bond type columns into ``node_feats`` V x h and ``edge_feats`` E x h, and
``EmbeddedChempropBlock``, the same embedding fused into the D-MPNN initial gather
(SURVEY §8(f) row 2).

``GraphEmbedding`` keeps the reference's module tree (``node`` / ``edge`` ``nn.EmbeddingBag``, so the
``state_dict`` keys match).  On a ROCm device without autograd its forward is the ``nt_embed_bag``
kernel; when gradients are needed it runs ``nn.EmbeddingBag`` itself (device ops) so the tables
train exactly as in the reference.  On the CPU it is the reference module unchanged (it is the
featurisation step ahead of the hot path, not the hot path).

``EmbeddedChempropBlock(embedding, block)`` computes ``block(embedding(G))`` — a drop-in for that
pair of modules in a ``TensorDictSequential`` — and, for inference on the device, runs
``nt_dmpnn_init_embed``: ``H0 = Xv[src] + Xe`` straight from the type indices and the two tables,
so the V x h / E x h embedded matrices are never written nor read back.  Bit-identical to the
unfused pair.
"""
from __future__ import annotations

import weakref

import torch
import torch.nn as nn

from notorch_amd import kernels as K
from notorch_amd._lib import NT_ACT_IDENTITY
from notorch_amd.data.models.graph import types_in_range
from notorch_amd.data.synth import DEFAULT_NUM_ATOM_TYPES, DEFAULT_NUM_BOND_TYPES
from notorch_amd.nn.gnn import _engine
from notorch_amd.nn.gnn.chemprop import ChempropBlock
from notorch_amd.nn.residual import Residual

DEFAULT_HIDDEN_DIM = 256  # notorch/conf.py


def _plain_bag(bag: nn.EmbeddingBag) -> bool:
    """The kernel covers the default EmbeddingBag configuration GraphEmbedding builds."""
    return (bag.mode == "sum" and bag.max_norm is None and bag.padding_idx is None
            and not bag.scale_grad_by_freq and not bag.include_last_offset)


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

    def _use_kernel(self, G) -> bool:
        w = self.node.weight
        needs_grad = torch.is_grad_enabled() and (w.requires_grad or self.edge.weight.requires_grad)
        return (w.device.type == "cuda" and not needs_grad and G.node_feats.dim() == 2
                and G.edge_feats.dim() == 2 and _plain_bag(self.node) and _plain_bag(self.edge))

    def forward(self, G):
        if self._use_kernel(G):
            nt_, et_ = G.node_feats.contiguous(), G.edge_feats.contiguous()
            ok = types_in_range(getattr(G, "_nt_layout", None), nt_, et_, self.num_node_types,
                                self.num_edge_types)
            if ok is False:
                raise IndexError("type index out of range for the embedding tables")
            Xv = K.embed_bag(self.node.weight.detach(), nt_, validate=ok is None)
            Xe = K.embed_bag(self.edge.weight.detach(), et_, validate=ok is None)
            return G.update(node_feats=Xv, edge_feats=Xe)
        return G.update(node_feats=self.node(G.node_feats), edge_feats=self.edge(G.edge_feats))

    @property
    def num_node_types(self) -> int:
        return self.node.num_embeddings

    @property
    def num_edge_types(self) -> int:
        return self.edge.num_embeddings


class EmbeddedChempropBlock(nn.Module):
    """``block(embedding(G))`` with the embedding fused into the block's initial gather."""

    def __init__(self, embedding: GraphEmbedding, block: ChempropBlock, fuse: bool = True):
        super().__init__()
        self.embedding = embedding
        self.block = block
        self.fuse = fuse  # False: GraphEmbedding kernel, then the block (same bytes out)

    def forward(self, G):
        emb, blk = self.embedding, self.block
        needs_grad = torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
        fusable = (
            self.fuse
            and G.node_feats.device.type == "cuda"
            and not needs_grad
            and emb._use_kernel(G)
            and emb.node.weight.dtype == emb.edge.weight.dtype
            and not any(l.training and l.update[1].p > 0 for l in blk._chemprop_layers())  # dropout
        )
        layers = blk._chemprop_layers()
        codes = [_engine.layer_act(l.act) for l in layers]
        if not fusable or any(c is None for c in codes) or len(set(codes)) > 1:
            return blk(emb(G))  # the block takes generic / mixed activations layer by layer
        if any(l.linear.weight.dtype != emb.node.weight.dtype for l in layers):
            raise RuntimeError("embedding tables and layer weights must share one dtype")
        act = codes[0] if codes else (NT_ACT_IDENTITY, 0.0)
        residual = bool(layers) and isinstance(blk.layers[0], Residual)
        # the layout needs V: give dst_layout a graph whose node_feats has V rows (the type matrix)
        lay = _engine.dst_layout(G)
        node_types, edge_types = G.node_feats.contiguous(), G.edge_feats.contiguous()
        seen = getattr(lay, "embed_checked", None)
        # the check is against these table sizes: a smaller table must re-validate the indices
        key = (node_types._version, edge_types._version, emb.node.num_embeddings, emb.edge.num_embeddings)
        validate = not (
            seen is not None and seen[0]() is node_types and seen[1]() is edge_types and seen[2] == key
        )
        if validate:  # the collate's host statistics answer without a device -> host sync
            ok = types_in_range(lay, node_types, edge_types, emb.node.num_embeddings, emb.edge.num_embeddings)
            if ok is False:
                raise IndexError("type index out of range for the embedding tables")
            validate = ok is None
        node, H = _engine.block_forward_embedded(
            emb.node.weight.detach(), node_types, emb.edge.weight.detach(), edge_types,
            G.edge_index[0].contiguous(), G.rev_index.contiguous(), lay,
            [l.linear.weight for l in layers], [l.linear.bias for l in layers], act, blk.reduce,
            residual, validate=validate,
        )
        # type indices validated for these tensors: no host sync on the next call
        lay.embed_checked = (weakref.ref(node_types), weakref.ref(edge_types), key)
        return G.update(node_feats=node, edge_feats=H)
