"""``ChempropLayer`` / ``ChempropBlock`` — drop-in replacements for
``notorch/nn/gnn/chemprop.py:13-88`` whose forward runs on the notorch_amd HIP kernels.

Same constructor signatures, attribute names, module tree and therefore ``state_dict`` keys
(``layers.{i}.module.update.0.{weight,bias}`` with ``residual=True``, ``layers.{i}.update.0.*``
without; one shared layer object repeated when ``shared=True``, chemprop.py:65-73), same
``forward(G) -> G.update(node_feats=..., edge_feats=...)`` contract (chemprop.py:81-88).

Differences by design:

* the forward runs only on ROCm device tensors; a CPU graph raises ``RuntimeError`` (there is no
  CPU fallback — the CPU restatement lives in ``oracle/`` and is test-only);
* ``dropout > 0`` in training mode draws its mask from a counter-based hash on the device
  (``nt_dropout_residual``) seeded from torch's default generator, not from torch's Philox stream:
  same distribution and scaling as ``nn.Dropout`` (keep with probability 1 - p, scale 1 / (1 - p)),
  different draws;
* ``act`` may be any activation module (chemprop.py:17,24,37).  ReLU, Identity, LeakyReLU, ELU,
  GELU, SiLU, Tanh and Sigmoid are fused into the kernels; any other module (e.g. ``nn.PReLU``,
  whose parameters train) runs as its own elementwise op between the segment-reduce and update
  kernels (``_engine.block_forward_layerwise``).
"""
from __future__ import annotations

from collections import OrderedDict

import torch
import torch.nn as nn
from torch import Tensor

from notorch_amd import kernels as K
from notorch_amd._lib import NT_ACT_IDENTITY
from notorch_amd.nn.gnn import _engine
from notorch_amd.nn.residual import Residual

Reduction = str  # Literal["mean", "sum", "min", "max"]  (notorch/types.py:57)
_REDUCTIONS = ("mean", "sum", "min", "max")


def _check_reduce(reduce: str) -> str:
    if reduce not in _REDUCTIONS:
        raise ValueError(f"reduce must be one of {_REDUCTIONS}, got {reduce!r}")
    return reduce


def _dropout(layers: list["ChempropLayer"]):
    """(p, seed) when the update's Dropout is active (training mode, p > 0; chemprop.py:26), else None."""
    ps = {float(l.update[1].p) for l in layers if l.training and l.update[1].p > 0}
    if not ps:
        return None
    if len(ps) > 1 or any(not l.training for l in layers):
        raise NotImplementedError("layers with different dropout settings are not supported")
    return ps.pop(), _engine.draw_dropout_seed()


class ChempropLayer(nn.Module):
    """One bond-message update (chemprop.py:13-46)."""

    def __init__(
        self,
        hidden_dim: int,
        act: type[nn.Module] = nn.ReLU,
        bias: bool = True,
        dropout: float = 0.0,
        reduce: Reduction = "sum",
    ):
        super().__init__()
        self.act = act()
        self.reduce = _check_reduce(reduce)
        self.update = nn.Sequential(nn.Linear(hidden_dim, hidden_dim, bias), nn.Dropout(dropout))
        self._csr_cache: "OrderedDict[int, tuple]" = OrderedDict()

    @property
    def linear(self) -> nn.Linear:
        return self.update[0]

    def _csr(self, edge_index: Tensor, rev_index: Tensor, V: int):
        key = id(edge_index)
        hit = self._csr_cache.get(key)
        if hit is not None and hit[0] is edge_index and hit[1] == V:
            return hit[2], hit[3]
        _engine._validate_indices(edge_index, rev_index, V)
        seg_ptr, perm = K.csr_build(edge_index[1].contiguous(), V, check_bounds=False)
        self._csr_cache[key] = (edge_index, V, seg_ptr, perm)
        while len(self._csr_cache) > 4:
            self._csr_cache.popitem(last=False)
        return seg_ptr, perm

    def forward(self, edge_feats: Tensor, node_feats: Tensor, edge_index: Tensor, rev_index: Tensor) -> Tensor:
        """U = Dropout(Linear(S[src] - act(H)[rev])), S = scatter(act(H), dst) — no residual here."""
        drop = _dropout([self])
        V = len(node_feats)
        act = _engine.layer_act(self.act)
        if drop is not None or act is None or (
                torch.is_grad_enabled() and (edge_feats.requires_grad or self.linear.weight.requires_grad)):
            # training through a standalone layer (or an activation without a kernel code): route
            # through the block function with depth 1 and no residual (it returns H_1 = U)
            lay = _engine.DeviceLayout(*self._csr(edge_index, rev_index, V), edge_index=edge_index, validated=True)
            Xv = torch.zeros(V, edge_feats.shape[1], device=edge_feats.device, dtype=edge_feats.dtype)
            # H0 = Xv[src] + Xe = edge_feats exactly (adding +0.0)
            if act is None:
                act_params = list(self.act.parameters())
                _, H = _engine.LayerwiseBlockFunction.apply(
                    Xv, edge_feats, edge_index, rev_index.contiguous(), lay, [(self.act, None)], [drop],
                    self.reduce, False, 1, len(act_params), self.linear.weight, self.linear.bias, *act_params,
                )
                return H
            _, H = _engine.ChempropBlockFunction.apply(
                Xv, edge_feats, edge_index, rev_index.contiguous(), lay, self.act, act, self.reduce,
                False, 1, drop, self.linear.weight, self.linear.bias,
            )
            return H
        seg_ptr, perm = self._csr(edge_index, rev_index, V)
        H = edge_feats.contiguous()
        S = K.segment_reduce(H, seg_ptr, perm, V, reduce=self.reduce, act=act)
        Wp = K.pack_weights(self.linear.weight.detach())
        b = None if self.linear.bias is None else self.linear.bias.detach()
        return K.dmpnn_update(
            H, S, edge_index[0].contiguous(), rev_index.contiguous(), Wp, b, residual=False, act=act
        )

    def extra_repr(self):
        return f"(reduce): {self.reduce}"


class ChempropBlock(nn.Module):
    """``depth`` bond-message layers + final node scatter (chemprop.py:49-88)."""

    def __init__(
        self,
        hidden_dim: int = 256,
        act: type[nn.Module] = nn.ReLU,
        bias: bool = True,
        dropout: float = 0.0,
        depth: int = 3,
        residual: bool = True,
        shared: bool = False,
        reduce: Reduction = "sum",
    ):
        super().__init__()
        if shared:
            layers = [ChempropLayer(hidden_dim, act, bias, dropout, reduce)] * depth
        else:
            layers = [ChempropLayer(hidden_dim, act, bias, dropout, reduce) for _ in range(depth)]
        if residual:
            layers = [Residual(layer) for layer in layers]
        self.layers = nn.ModuleList(layers)
        self.hidden_dim = hidden_dim
        self.reduce = _check_reduce(reduce)
        self.residual = residual

    @property
    def depth(self) -> int:
        return len(self.layers)

    def _chemprop_layers(self) -> list[ChempropLayer]:
        return [m.module if isinstance(m, Residual) else m for m in self.layers]

    def forward(self, G):
        Xv, Xe = G.node_feats, G.edge_feats
        if Xv.device.type != "cuda":
            raise RuntimeError(
                "notorch_amd.ChempropBlock runs on ROCm devices only (no CPU fallback); "
                f"got node_feats on '{Xv.device}'"
            )
        if Xv.dim() != 2 or Xe.dim() != 2 or Xv.shape[1] != Xe.shape[1]:
            raise RuntimeError(
                f"node_feats {tuple(Xv.shape)} and edge_feats {tuple(Xe.shape)} must share the "
                "hidden dimension (chemprop.py:83)"
            )
        layers = self._chemprop_layers()
        if Xv.dtype != Xe.dtype or any(l.linear.weight.dtype != Xv.dtype for l in layers):
            # what nn.Linear / the Xv[src] + Xe add would raise on mixed dtypes in the reference
            raise RuntimeError(
                f"node_feats ({Xv.dtype}), edge_feats ({Xe.dtype}) and the layer weights must share "
                "one dtype (float32, or bfloat16 after block.to(torch.bfloat16))"
            )
        residual = bool(layers) and isinstance(self.layers[0], Residual)
        lay = _engine.dst_layout(G)
        Xv = Xv.contiguous()
        Xe = Xe.contiguous()
        rev = G.rev_index.contiguous()
        weights = [layer.linear.weight for layer in layers]
        biases = [layer.linear.bias for layer in layers]
        needs_grad = torch.is_grad_enabled() and (
            Xv.requires_grad or Xe.requires_grad or any(p.requires_grad for p in self.parameters())
        )
        codes = [_engine.layer_act(layer.act) for layer in layers]
        dps = [float(l.update[1].p) if l.training and l.update[1].p > 0 else None for l in layers]
        uniform = all(c is not None for c in codes) and len(set(codes)) <= 1 and len(set(dps)) <= 1
        if not uniform:
            seed = _engine.draw_dropout_seed() if any(p is not None for p in dps) else 0
            drops = [None if p is None else (p, seed) for p in dps]  # disjoint per-layer offsets
            # an activation without a kernel code, or layers that differ in activation / dropout:
            # the layer-by-layer device path (_engine.block_forward_layerwise)
            acts = [(layer.act, c) for layer, c in zip(layers, codes)]
            if needs_grad:
                # the activation modules' parameters (nn.PReLU's slope ...) train through the
                # Function's recompute backward; shared modules contribute their tensors once
                act_params = list({id(p): p for l in layers for p in l.act.parameters()}.values())
                node, H = _engine.LayerwiseBlockFunction.apply(
                    Xv, Xe, G.edge_index, rev, lay, acts, drops, self.reduce, residual, len(layers),
                    len(act_params), *weights, *biases, *act_params,
                )
            else:
                node, H = _engine.block_forward_layerwise(
                    Xv, Xe, G.edge_index[0].contiguous(), rev, lay, acts, weights, biases, drops,
                    self.reduce, residual,
                )
            return G.update(node_feats=node, edge_feats=H)
        drop = _dropout(layers)
        act = codes[0] if codes else (NT_ACT_IDENTITY, 0.0)
        if needs_grad:
            node, H = _engine.ChempropBlockFunction.apply(
                Xv, Xe, G.edge_index, rev, lay, layers[0].act if layers else nn.Identity(), act,
                self.reduce, residual, len(layers), drop, *weights, *biases,
            )
        else:
            src = G.edge_index[0].contiguous()
            node, H, _ = _engine.block_forward(
                Xv, Xe, src, rev, lay, weights, biases, act, self.reduce, residual, drop=drop
            )
        return G.update(node_feats=node, edge_feats=H)
