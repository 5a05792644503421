"""GPU parity of the layer-by-layer device path (_engine.block_forward_layerwise): activations with no
kernel code (the reference takes any nn.Module class, chemprop.py:17,24,37) and blocks whose layers
differ in activation.  Oracle: oracle/dmpnn_ref.py (chemprop.py:28-43, :81-88; residual.py:27-28)
with the same activation callables; fp32 contract FP32_NORM_TOL."""
import pytest
import torch
import torch.nn as nn

from helpers import FP32_NORM_TOL, assert_parity
from oracle import dmpnn_ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _graph(n=40, seed=0, rev_offset="nodes"):
    from notorch_amd.data.synth import make_batch

    return make_batch("qm9", n, seed=seed).collate(rev_offset)


def _ref_layers(G, Xv, Xe, Ws, bs, acts, reduce="sum", residual=True):
    src, dst = G.edge_index
    H = Xv[src] + Xe
    for W, b, act in zip(Ws, bs, acts):
        U = dmpnn_ref.chemprop_layer(H, Xv, G.edge_index, G.rev_index, W, b, act, reduce)
        H = H + U if residual else U
    return dmpnn_ref.scatter(H, dst, G.num_nodes, reduce), H


@pytest.mark.parametrize("act,reduce,residual", [
    (nn.Softplus, "sum", True), (nn.Mish, "mean", False), (nn.Hardswish, "max", True),
])
def test_generic_activation_block(act, reduce, residual):
    from notorch_amd.nn import ChempropBlock

    G = _graph(48, seed=2)
    torch.manual_seed(0)
    h = 96
    Xv, Xe = torch.randn(G.num_nodes, h), torch.randn(G.num_edges, h)
    blk = ChempropBlock(hidden_dim=h, act=act, depth=3, reduce=reduce, residual=residual).eval()
    Ws, bs = dmpnn_ref.block_params(blk)
    ref_n, ref_e = _ref_layers(G, Xv, Xe, Ws, bs, [act()] * 3, reduce, residual)
    with torch.no_grad():
        out = blk.to(DEV)(G.update(node_feats=Xv, edge_feats=Xe).to(DEV))
    assert_parity(out.edge_feats, ref_e, FP32_NORM_TOL, "edge")
    assert_parity(out.node_feats, ref_n, FP32_NORM_TOL, "node")


def test_mixed_per_layer_activations():
    from notorch_amd.nn import ChempropBlock

    G = _graph(40, seed=4, rev_offset="edges")
    torch.manual_seed(1)
    h = 64
    Xv, Xe = torch.randn(G.num_nodes, h), torch.randn(G.num_edges, h)
    blk = ChempropBlock(hidden_dim=h, depth=3).eval()
    mods = [nn.ReLU(), nn.Tanh(), nn.Softplus()]
    for m, a in zip(blk._chemprop_layers(), mods):
        m.act = a
    Ws, bs = dmpnn_ref.block_params(blk)
    ref_n, ref_e = _ref_layers(G, Xv, Xe, Ws, bs, mods)
    with torch.no_grad():
        out = blk.to(DEV)(G.update(node_feats=Xv, edge_feats=Xe).to(DEV))
    assert_parity(out.edge_feats, ref_e, FP32_NORM_TOL, "edge")
    assert_parity(out.node_feats, ref_n, FP32_NORM_TOL, "node")


def test_generic_activation_gradients():
    """Kernel forward + recompute backward: gradients of Xv, Xe and every weight / bias against fp64
    oracle autograd (smooth activation: no ReLU sign-flip floor)."""
    from notorch_amd.nn import ChempropBlock

    G = _graph(24, seed=5)
    torch.manual_seed(2)
    h = 48
    Xv, Xe = torch.randn(G.num_nodes, h), torch.randn(G.num_edges, h)
    blk = ChempropBlock(hidden_dim=h, act=nn.Softplus, depth=2).train()
    Ws, bs = dmpnn_ref.block_params(blk)
    Xv64, Xe64 = Xv.double().requires_grad_(), Xe.double().requires_grad_()
    W64 = [w.double().requires_grad_() for w in Ws]
    b64 = [b.double().requires_grad_() for b in bs]
    n64, e64 = _ref_layers(G, Xv64, Xe64, W64, b64, [nn.Softplus()] * 2)
    (n64.sum() + (e64 ** 2).mean()).backward()

    blk = blk.to(DEV)
    Xv_d, Xe_d = Xv.to(DEV).requires_grad_(), Xe.to(DEV).requires_grad_()
    out = blk(G.update(node_feats=Xv_d, edge_feats=Xe_d).to(DEV))
    (out.node_feats.sum() + (out.edge_feats ** 2).mean()).backward()
    assert_parity(Xv_d.grad, Xv64.grad, FP32_NORM_TOL, "dXv")
    assert_parity(Xe_d.grad, Xe64.grad, FP32_NORM_TOL, "dXe")
    for i, m in enumerate(blk._chemprop_layers()):
        assert_parity(m.linear.weight.grad, W64[i].grad, FP32_NORM_TOL, f"dW{i}")
        assert_parity(m.linear.bias.grad, b64[i].grad, FP32_NORM_TOL, f"db{i}")


def test_standalone_layer_generic_activation():
    from notorch_amd.nn import ChempropLayer

    G = _graph(16, seed=6)
    torch.manual_seed(3)
    h = 32
    H, Xv = torch.randn(G.num_edges, h), torch.randn(G.num_nodes, h)
    layer = ChempropLayer(h, nn.SELU).eval()
    ref = dmpnn_ref.chemprop_layer(H, Xv, G.edge_index, G.rev_index, layer.linear.weight.detach(),
                                   layer.linear.bias.detach(), nn.SELU())
    with torch.no_grad():
        out = layer.to(DEV)(H.to(DEV), Xv.to(DEV), G.edge_index.to(DEV), G.rev_index.to(DEV))
    assert_parity(out, ref, FP32_NORM_TOL, "layer")


def test_prelu_slope_trains():
    """nn.PReLU's slope is a parameter of the activation module (the reference accepts any
    nn.Module class, chemprop.py:17,24): its gradient comes back through the layer-by-layer
    Function and matches fp64 oracle autograd, next to dXv, dXe and every dW / db."""
    from notorch_amd.nn import ChempropBlock

    G = _graph(24, seed=8)
    torch.manual_seed(4)
    h = 48
    Xv, Xe = torch.randn(G.num_nodes, h), torch.randn(G.num_edges, h)
    blk = ChempropBlock(hidden_dim=h, act=nn.PReLU, depth=2).train()
    for m in blk._chemprop_layers():
        nn.init.constant_(m.act.weight, 0.3)
    Ws, bs = dmpnn_ref.block_params(blk)
    Xv64, Xe64 = Xv.double().requires_grad_(), Xe.double().requires_grad_()
    W64 = [w.double().requires_grad_() for w in Ws]
    b64 = [b.double().requires_grad_() for b in bs]
    acts64 = [nn.PReLU(init=0.3).double() for _ in range(2)]
    n64, e64 = _ref_layers(G, Xv64, Xe64, W64, b64, acts64)
    (n64.sum() + (e64 ** 2).mean()).backward()

    blk = blk.to(DEV)
    Xv_d, Xe_d = Xv.to(DEV).requires_grad_(), Xe.to(DEV).requires_grad_()
    out = blk(G.update(node_feats=Xv_d, edge_feats=Xe_d).to(DEV))
    (out.node_feats.sum() + (out.edge_feats ** 2).mean()).backward()
    assert_parity(Xv_d.grad, Xv64.grad, FP32_NORM_TOL * 2, "dXv")
    assert_parity(Xe_d.grad, Xe64.grad, FP32_NORM_TOL * 2, "dXe")
    for i, m in enumerate(blk._chemprop_layers()):
        assert m.act.weight.grad is not None, f"PReLU slope of layer {i} got no gradient"
        assert_parity(m.act.weight.grad, acts64[i].weight.grad, FP32_NORM_TOL * 2, f"dslope{i}")
        assert_parity(m.linear.weight.grad, W64[i].grad, FP32_NORM_TOL * 2, f"dW{i}")


def test_rrelu_training_backward_replays_forward_draws():
    """A stochastic activation (nn.RReLU in training mode) draws its slopes once in the forward; the
    recompute backward replays the same draws, so the gradient is that of the function the forward
    computed: check d(sum H_d)/dXe against torch autograd on the same forward with the same RNG."""
    from notorch_amd.nn import ChempropBlock
    from notorch_amd.nn.gnn import _engine

    G = _graph(16, seed=9, rev_offset="edges")
    torch.manual_seed(5)
    h = 32
    Xv, Xe = torch.randn(G.num_nodes, h), torch.randn(G.num_edges, h)
    blk = ChempropBlock(hidden_dim=h, act=nn.RReLU, depth=2).train().to(DEV)
    Gd = G.update(node_feats=Xv, edge_feats=Xe).to(DEV)
    Xe_d = Gd.edge_feats.clone().requires_grad_()
    torch.cuda.manual_seed(11)
    out = blk(Gd.update(edge_feats=Xe_d))
    out.edge_feats.sum().backward()
    # the same forward in device torch ops from the same RNG state
    Xe_t = Gd.edge_feats.clone().requires_grad_()
    layers = blk._chemprop_layers()
    torch.cuda.manual_seed(11)
    _, H = _engine._torch_block_layerwise(Gd.node_feats, Xe_t, Gd.edge_index, Gd.rev_index,
                                          [l.linear.weight for l in layers], [l.linear.bias for l in layers],
                                          [l.act for l in layers], "sum", True, [None, None])
    assert_parity(out.edge_feats.detach(), H.detach(), FP32_NORM_TOL, "H (same draws)")
    H.sum().backward()
    assert_parity(Xe_d.grad, Xe_t.grad, FP32_NORM_TOL, "dXe")
