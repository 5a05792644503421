"""Training-mode dropout of the layer update (chemprop.py:26 `Dropout(p)` inside `update`, applied at
:42 before residual.py:28's add), on the nt_dropout_residual kernel.

The mask comes from a counter-based hash on the device, not from torch's Philox stream, so draws
cannot equal the reference's; what is pinned instead:
* the kernel: exact values (0 or Y / (1 - p), plus base), keep rate 1 - p within 5 sigma,
  determinism in (seed, offset), independence of neighbouring offsets, p = 0 / p = 1 limits;
* the block: forward and every gradient equal the fp64 oracle (oracle/dmpnn_ref.chemprop_block
  with the same masks, recovered by running the kernel on ones) within the fp32 contract;
* the seed is drawn from torch's default generator: torch.manual_seed reproduces a training step.
"""
import math

import pytest
import torch
import torch.nn as nn

from helpers import assert_parity
from oracle import dmpnn_ref

pytestmark = pytest.mark.gpu

DEV = "cuda"
TOL = 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n", [1 << 20, 999_997])  # 16-B pieces, scalar tail path
def test_dropout_kernel_values_and_rate(dtype, n):
    from notorch_amd import kernels as K

    p = 0.3
    g = torch.Generator(device=DEV).manual_seed(0)
    Y = torch.randn(n, device=DEV, generator=g).to(dtype)
    base = torch.randn(n, device=DEV, generator=g).to(dtype)
    out = K.dropout_residual(Y, p, seed=1234, offset=7, base=base)
    mask = K.dropout_residual(torch.ones_like(Y), p, seed=1234, offset=7)
    scale = 1.0 / (1.0 - p)
    kept = mask != 0
    assert torch.all((mask == 0) | (mask == torch.tensor(scale, dtype=torch.float32).to(dtype)))
    ref = (base.float() + torch.where(kept, Y.float() * scale, 0.0)).to(dtype)
    if dtype == torch.float32:
        assert torch.equal(out, ref)
    else:  # one rounding of the fp32 value
        assert_parity(out.float(), ref.float(), 2.0 ** -8, "bf16 dropout")
    rate = kept.float().mean().item()
    assert abs(rate - (1 - p)) < 5 * math.sqrt(p * (1 - p) / n), rate
    # deterministic in (seed, offset); another seed or a shifted offset gives another mask
    assert torch.equal(K.dropout_residual(Y, p, seed=1234, offset=7, base=base), out)
    m2 = K.dropout_residual(torch.ones_like(Y), p, seed=1235, offset=7) != 0
    m3 = K.dropout_residual(torch.ones_like(Y), p, seed=1234, offset=8) != 0
    for other in (m2, m3):
        agree = (other == kept).float().mean().item()
        assert abs(agree - (p * p + (1 - p) ** 2)) < 0.01, agree
    # the shifted-offset mask is the same stream moved by one element
    assert torch.equal(m3[:-1], kept[1:])


def test_dropout_kernel_limits():
    from notorch_amd import kernels as K

    Y = torch.randn(4096, device=DEV)
    base = torch.randn(4096, device=DEV)
    assert torch.equal(K.dropout_residual(Y, 0.0, 5, base=base), base + Y)
    assert torch.equal(K.dropout_residual(Y, 1.0, 5, base=base), base)
    assert torch.equal(K.dropout_residual(Y, 1.0, 5), torch.zeros_like(Y))
    with pytest.raises(Exception, match="probability"):
        K.dropout_residual(Y, 1.5, 5)


def _masks(seed, p, E, h, depth):
    from notorch_amd import kernels as K
    from notorch_amd.nn.gnn import _engine

    ones = torch.ones(E, h, device=DEV)
    return [K.dropout_residual(ones, p, seed, _engine.dropout_offset(l, E, h)).double().cpu()
            for l in range(depth)]


@pytest.mark.parametrize("reduce,residual", [("sum", True), ("mean", True), ("sum", False), ("max", True)])
def test_block_dropout_forward_and_grads(reduce, residual):
    from notorch_amd.data.synth import make_batch
    from notorch_amd.nn import ChempropBlock
    from notorch_amd.nn.gnn import _engine

    G = make_batch("qm9", 24, seed=4).collate("nodes")
    h, depth, p = 48, 3, 0.25
    torch.manual_seed(0)
    Xv = nn.EmbeddingBag(42, h, mode="sum")(G.node_feats).detach()
    Xe = nn.EmbeddingBag(13, h, mode="sum")(G.edge_feats).detach()
    torch.manual_seed(1)
    blk = ChempropBlock(h, depth=depth, dropout=p, reduce=reduce, residual=residual).to(DEV).train()

    torch.manual_seed(99)
    seed = _engine.draw_dropout_seed()
    masks = _masks(seed, p, G.num_edges, h, depth)
    assert all(0.6 < (m != 0).double().mean().item() < 0.9 for m in masks)

    torch.manual_seed(99)  # the block draws the same seed
    Xv_d, Xe_d = Xv.to(DEV).requires_grad_(True), Xe.to(DEV).requires_grad_(True)
    out = blk(G.update(node_feats=Xv_d, edge_feats=Xe_d).to(DEV))
    wts = torch.linspace(-1, 1, h, device=DEV)
    (out.node_feats.pow(2).sum() + (out.edge_feats * wts).sum()).backward()

    Ws, bs = dmpnn_ref.block_params(blk)
    Ws = [W.double().requires_grad_(True) for W in Ws]
    bs = [b.double().requires_grad_(True) for b in bs]
    Xv_r, Xe_r = Xv.double().requires_grad_(True), Xe.double().requires_grad_(True)
    n_r, e_r = dmpnn_ref.chemprop_block(Xv_r, Xe_r, G.edge_index, G.rev_index, Ws, bs, residual=residual,
                                        reduce=reduce, dropout_masks=masks)
    (n_r.pow(2).sum() + (e_r * wts.double().cpu()).sum()).backward()

    assert_parity(out.node_feats, n_r, TOL, "node")
    assert_parity(out.edge_feats, e_r, TOL, "edge")
    assert_parity(Xv_d.grad, Xv_r.grad, TOL, "dXv")
    assert_parity(Xe_d.grad, Xe_r.grad, TOL, "dXe")
    for l, layer in enumerate(blk._chemprop_layers()):
        assert_parity(layer.linear.weight.grad, Ws[l].grad, TOL, f"dW[{l}]")
        assert_parity(layer.linear.bias.grad, bs[l].grad, TOL, f"db[{l}]")


def test_dropout_eval_and_no_grad_training():
    """eval(): no dropout (the inference path); train() under no_grad still drops (nn.Dropout does)."""
    from notorch_amd.data.synth import make_batch
    from notorch_amd.nn import ChempropBlock

    G = make_batch("qm9", 8, seed=5).collate("nodes")
    h = 32
    torch.manual_seed(0)
    Xv = nn.EmbeddingBag(42, h, mode="sum")(G.node_feats).detach()
    Xe = nn.EmbeddingBag(13, h, mode="sum")(G.edge_feats).detach()
    Gd = G.update(node_feats=Xv, edge_feats=Xe).to(DEV)
    torch.manual_seed(1)
    blk = ChempropBlock(h, depth=2, dropout=0.5).to(DEV)
    plain = ChempropBlock(h, depth=2, dropout=0.0).to(DEV)
    plain.load_state_dict(blk.state_dict())
    with torch.no_grad():
        ev = blk.eval()(Gd).edge_feats
        assert torch.equal(ev, plain.eval()(Gd).edge_feats)
        torch.manual_seed(3)
        t1 = blk.train()(Gd).edge_feats
        torch.manual_seed(3)
        t2 = blk(Gd).edge_feats
        t3 = blk(Gd).edge_feats
    assert torch.equal(t1, t2) and not torch.equal(t1, t3) and not torch.equal(t1, ev)


def test_standalone_layer_dropout_matches_oracle():
    from notorch_amd.data.synth import make_batch
    from notorch_amd.nn import ChempropLayer
    from notorch_amd.nn.gnn import _engine

    G = make_batch("qm9", 8, seed=6).collate("nodes")
    h, p = 32, 0.4
    torch.manual_seed(0)
    H = torch.randn(G.num_edges, h)
    layer = ChempropLayer(h, dropout=p).to(DEV).train()
    torch.manual_seed(7)
    seed = _engine.draw_dropout_seed()
    (mask,) = _masks(seed, p, G.num_edges, h, 1)
    ei, rev = G.edge_index.clone(), G.rev_index.clone()
    torch.manual_seed(7)
    with torch.no_grad():
        got = layer(H.to(DEV), torch.zeros(G.num_nodes, h, device=DEV), ei.to(DEV), rev.to(DEV))
    W = layer.linear.weight.detach().double().cpu()
    b = layer.linear.bias.detach().double().cpu()
    ref = dmpnn_ref.chemprop_layer(H.double(), torch.zeros(G.num_nodes, h, dtype=torch.float64),
                                   ei, rev, W, b) * mask
    assert_parity(got, ref, TOL, "layer dropout")
