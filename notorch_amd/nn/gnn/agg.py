"""Graph readouts (reference ``notorch/nn/gnn/agg.py:15-47``) on the segment-reduce kernel.

``Sum`` / ``Mean`` / ``Max`` reduce ``G.node_feats`` over the nodes of each molecule
(``batch_node_index``, ``dim_size=len(G)``) with torch_scatter semantics: mean divides by
``max(count, 1)``, an empty molecule reads 0 for every reduction.  ``Min`` is added for
completeness of the ``Reduction`` domain (notorch/types.py:57).

``Gated`` and ``SDPAttention`` (agg.py:50-86) weight the nodes of each molecule
by a per-molecule softmax of a node score (``nt_node_scores`` then ``nt_softmax_pool``).  ``Gated``
uses alpha as the (V, 1) node weight agg.py:59-61 evidently means: the reference's extra
``.unsqueeze(1)`` turns alpha into (V, 1, 1), which broadcasts against (V, d) into a (V, V, d) tensor
and returns (b, V, d) — O(b V d) memory and not a readout.  This is the one documented divergence.
Training through them runs the kernel backward (``nt_softmax_pool_backward``): the gradients of X,
of Gated's ``a`` and of SDPAttention's query Q.
"""
from __future__ import annotations

from abc import abstractmethod
from math import sqrt

import torch
import torch.nn as nn
from torch import Tensor

from notorch_amd import kernels as K
from notorch_amd.nn.gnn import _engine

DEFAULT_HIDDEN_DIM = 256  # notorch/conf.py


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
            X.contiguous(), mol_ptr, mol_perm, len(G), self.reduce, G.batch_node_index,
            _engine.mol_chunks(G, mol_ptr),
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


def _softmax_pool_torch(X: Tensor, scores: Tensor, bni: Tensor, B: int) -> Tensor:
    """The same readout in device ops (autograd path): scatter_softmax + scatter_sum."""
    idx = bni.view(-1)
    mx = torch.full((B,), float("-inf"), dtype=scores.dtype, device=scores.device)
    mx = mx.scatter_reduce(0, idx, scores, reduce="amax", include_self=True)
    rec = (scores - mx[idx]).exp()
    z = torch.zeros(B, dtype=scores.dtype, device=scores.device).scatter_add(0, idx, rec)
    alpha = (rec / z[idx]).unsqueeze(1).to(X.dtype)
    out = torch.zeros(B, X.shape[1], dtype=X.dtype, device=X.device)
    return out.scatter_add(0, idx.view(-1, 1).expand_as(X), alpha * X)


class SoftmaxPoolFunction(torch.autograd.Function):
    """nt_node_scores + nt_softmax_pool with the kernel backward (nt_softmax_pool_backward).
    key: Gated's a.weight (1 x d) with bias (1,) or None; SDPAttention's Q (b x d) with bias None."""

    @staticmethod
    def forward(ctx, X, key, bias, sdpa, sqrt_key, mol_ptr, mol_perm, bni, B):
        if sdpa:
            scores = K.node_scores(X, Q=key.contiguous(), node_seg=bni.contiguous(), sqrt_key=sqrt_key)
        else:
            scores = K.node_scores(X, a=key.detach().reshape(-1).contiguous(),
                                   a_bias=None if bias is None else bias.detach())
        out = K.softmax_pool(X, scores, mol_ptr, mol_perm, B)
        ctx.save_for_backward(X, key, scores, out, bni)
        ctx.cfg = (sdpa, sqrt_key, mol_ptr, mol_perm, B, bias is not None)
        return out

    @staticmethod
    def backward(ctx, dout):
        X, key, scores, out, bni = ctx.saved_tensors
        sdpa, sqrt_key, mol_ptr, mol_perm, B, has_bias = ctx.cfg
        k = key.detach().contiguous() if sdpa else key.detach().reshape(-1).contiguous()
        dX, ds, P = K.softmax_pool_backward(
            X, scores, mol_ptr, mol_perm, bni.contiguous(), B, out, dout.contiguous().to(X.dtype),
            a=None if sdpa else k, Q=k if sdpa else None, sqrt_key=sqrt_key)
        if sdpa:
            dkey, dbias = (P / sqrt_key).to(key.dtype), None
        else:
            dkey = P.sum(0).reshape(key.shape).to(key.dtype)
            dbias = ds.sum().reshape(1).to(key.dtype) if has_bias else None
        return dX, dkey, dbias, None, None, None, None, None, None


class _AttentionReadout(Aggregation):
    def _pool(self, G, key, bias, sdpa, sqrt_key=1.0) -> Tensor:
        """Scores and softmax pool on the kernels; under autograd the kernel backward
        (SoftmaxPoolFunction) for X, the module's parameters and the SDPAttention query."""
        X = G.node_feats
        if X.device.type != "cuda":
            raise RuntimeError(
                f"notorch_amd.{type(self).__name__} runs on ROCm devices only; got '{X.device}'"
            )
        X = X.contiguous()
        B = len(G)
        mol_ptr, mol_perm = _engine.mol_layout(G)
        bni = G.batch_node_index
        if sdpa and (key.dim() != 2 or key.shape[1] != X.shape[1]):
            raise RuntimeError(f"Q must be b x {X.shape[1]}, got {tuple(key.shape)}")
        needs_grad = torch.is_grad_enabled() and (
            X.requires_grad or key.requires_grad or (bias is not None and bias.requires_grad))
        if needs_grad:
            return SoftmaxPoolFunction.apply(X, key, bias, sdpa, sqrt_key, mol_ptr, mol_perm, bni, B)
        with torch.no_grad():
            return SoftmaxPoolFunction.forward(_NoCtx(), X, key, bias, sdpa, sqrt_key, mol_ptr, mol_perm, bni, B)


class _NoCtx:
    """Context stand-in for the no-grad forward (nothing is saved)."""

    def save_for_backward(self, *a):
        pass


class Gated(_AttentionReadout):
    """agg.py:50-63: alpha = softmax over each molecule of a(x_v); out[g] = sum_v alpha_v x_v."""

    def __init__(self, input_dim: int = DEFAULT_HIDDEN_DIM):
        super().__init__()
        self.a = nn.Linear(input_dim, 1)

    def forward(self, G, **kwargs) -> Tensor:
        return self._pool(G, self.a.weight, self.a.bias, sdpa=False)


class SDPAttention(_AttentionReadout):
    """agg.py:66-86: scores = <Q[batch v], x_v> / sqrt(key_dim), softmax per molecule, weighted sum."""

    def __init__(self, key_dim: int = DEFAULT_HIDDEN_DIM):
        super().__init__()
        self.sqrt_key_dim = sqrt(key_dim)

    def forward(self, G, *, Q: Tensor, **kwargs) -> Tensor:
        return self._pool(G, Q, None, sdpa=True, sqrt_key=self.sqrt_key_dim)
