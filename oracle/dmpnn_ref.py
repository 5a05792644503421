"""CPU restatement of the reference D-MPNN forward (TEST INFRASTRUCTURE ONLY — see oracle/__init__).

Op for op, in the reference's order and on the same ATen kernels the reference dispatches to
(``index``, ``scatter_add_``, ``addmm``), so that on CPU it reproduces the reference's numbers:

* ``scatter``            torch_scatter 2.1.x ``scatter(src, index, dim=0, dim_size, reduce)``
                         (third-party; called at chemprop.py:39,86 and agg.py:27,36,45):
                         sum  = zeros(dim_size, h).scatter_add_(0, index.view(-1,1).expand_as(src), src)
                         mean = sum / count.clamp(min=1)
                         max/min: segment extreme, empty segment -> 0
* ``chemprop_layer``     notorch/nn/gnn/chemprop.py:28-43
* ``chemprop_block``     notorch/nn/gnn/chemprop.py:81-88 with Residual (notorch/nn/residual.py:27-28)
* ``readout``            notorch/nn/gnn/agg.py:23-47 (Sum / Mean / Max)
* ``readout_gated`` / ``readout_sdpa``   agg.py:50-86 (Gated / SDPAttention, scatter_softmax)
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import torch
from torch import Tensor


def scatter(src: Tensor, index: Tensor, dim_size: int, reduce: str = "sum") -> Tensor:
    """torch_scatter.scatter along dim 0 (torch_scatter/scatter.py: scatter_sum/mean/max/min)."""
    out = torch.zeros((dim_size,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    idx = index.view(-1, *([1] * (src.dim() - 1))).expand_as(src)
    if reduce == "sum":
        return out.scatter_add_(0, idx, src)
    if reduce == "mean":
        s = out.scatter_add_(0, idx, src)
        count = torch.zeros(dim_size, dtype=src.dtype, device=src.device).scatter_add_(
            0, index, torch.ones_like(index, dtype=src.dtype)
        )
        count = count.clamp(min=1).view(-1, *([1] * (src.dim() - 1)))
        return s / count
    if reduce in ("max", "min"):
        # torch_scatter's scatter_max/min leave empty segments at 0 (their C++ kernels fill the
        # untouched lowest()/max() sentinels with 0); include_self=False on a zero tensor matches.
        return out.scatter_reduce_(0, idx, src, reduce="amax" if reduce == "max" else "amin",
                                   include_self=False)
    raise ValueError(reduce)


def chemprop_layer(
    edge_feats: Tensor,
    node_feats: Tensor,
    edge_index: Tensor,
    rev_index: Tensor,
    weight: Tensor,
    bias: Optional[Tensor],
    act: Callable[[Tensor], Tensor] = torch.relu,
    reduce: str = "sum",
) -> Tensor:
    """chemprop.py:28-43 (Dropout in eval mode is the identity)."""
    src, dest = edge_index.unbind(0)
    edge_hiddens = act(edge_feats)                                                    # :37
    messages = edge_hiddens                                                           # :38
    node_messages = scatter(messages, dest, dim_size=len(node_feats), reduce=reduce)  # :39
    edge_messages = node_messages[src] - messages[rev_index]                          # :40
    return torch.nn.functional.linear(edge_messages, weight, bias)                    # :41 (:26)


def chemprop_block(
    node_feats: Tensor,
    edge_feats: Tensor,
    edge_index: Tensor,
    rev_index: Tensor,
    weights: Sequence[Tensor],
    biases: Sequence[Optional[Tensor]],
    act: Callable[[Tensor], Tensor] = torch.relu,
    residual: bool = True,
    reduce: str = "sum",
    dropout_masks: Optional[Sequence[Tensor]] = None,
) -> tuple[Tensor, Tensor]:
    """chemprop.py:81-88 -> (node_hiddens V x h, edge_hiddens E x h).  dropout_masks: per layer, the
    E x h factor nn.Dropout applied to the update in training mode (keep / (1 - p), chemprop.py:26)."""
    src, dest = edge_index.unbind(0)
    edge_hiddens = node_feats[src] + edge_feats                                       # :82-83
    for l, (W, b) in enumerate(zip(weights, biases)):                                 # :84
        out = chemprop_layer(edge_hiddens, node_feats, edge_index, rev_index, W, b, act, reduce)
        if dropout_masks is not None:
            out = out * dropout_masks[l]                                              # :26 Dropout
        edge_hiddens = edge_hiddens + out if residual else out                        # residual.py:28
    node_hiddens = scatter(edge_hiddens, dest, dim_size=len(node_feats), reduce=reduce)  # :86
    return node_hiddens, edge_hiddens


def readout(node_feats: Tensor, batch_node_index: Tensor, size: int, kind: str = "sum") -> Tensor:
    """agg.py:23-47: Sum / Mean / Max (+ Min) over molecules."""
    return scatter(node_feats, batch_node_index, dim_size=size, reduce=kind)


def scatter_softmax(src: Tensor, index: Tensor, dim_size: int) -> Tensor:
    """torch_scatter composite/softmax.py scatter_softmax along dim 0 (1-D scores):
    exp(src - max_g) / sum_g exp(src - max_g), the max and sum by scatter."""
    mx = scatter(src, index, dim_size, "max")
    rec = (src - mx[index]).exp()
    return rec / scatter(rec, index, dim_size, "sum")[index]


def readout_gated(node_feats: Tensor, batch_node_index: Tensor, size: int, a_weight: Tensor,
                  a_bias: Optional[Tensor]) -> Tensor:
    """agg.py:50-63 with alpha used as the (V, 1) node weight it evidently means: scores = a(x)
    (:59), alpha = scatter_softmax(scores) (:60), out = scatter_sum(alpha * x) (:61).  The
    reference's extra .unsqueeze(1) broadcasts (V,1,1) * (V,d) to (V,V,d); that shape
    bug is not restated."""
    scores = torch.nn.functional.linear(node_feats, a_weight, a_bias).squeeze(-1)
    alpha = scatter_softmax(scores, batch_node_index, size).unsqueeze(1)
    return scatter(alpha * node_feats, batch_node_index, size, "sum")


def readout_sdpa(node_feats: Tensor, batch_node_index: Tensor, size: int, Q: Tensor,
                 sqrt_key_dim: float) -> Tensor:
    """agg.py:66-86: scores = <Q[batch v], x_v> / sqrt(key_dim); softmax per molecule; weighted sum."""
    scores = torch.einsum("vd,vd->v", Q[batch_node_index], node_feats) / sqrt_key_dim
    alpha = scatter_softmax(scores, batch_node_index, size).unsqueeze(1)
    return scatter(alpha * node_feats, batch_node_index, size, "sum")


def block_params(module) -> tuple[list, list]:
    """(weights, biases) of a ChempropBlock-shaped module (layers[i](.module).update[0])."""
    ws, bs = [], []
    for m in module.layers:
        layer = getattr(m, "module", m)
        lin = layer.update[0]
        ws.append(lin.weight.detach().cpu())
        bs.append(None if lin.bias is None else lin.bias.detach().cpu())
    return ws, bs
