"""GPU parity of the fp32 layer kernel on the two-part fp16 split (update_fk_kernel): 128-row balanced
tile plans (h <= 384, relu layers with a sum aggregation), 64-row plans for the other variants and the
column-chunked h > 384 path, every aggregation variant, the amax chain that scales the split, operands
far from unit magnitude, hidden sizes beyond 512 (the reference accepts any hidden_dim,
chemprop.py:54), and the kernels' row-capacity check.  Oracle: fp64 evaluation of chemprop.py:36-43 / residual.py:27-28 and
the CPU scatter of the kernel's own H_out (chemprop.py:37-39, :86); fp32 contract FP32_NORM_TOL."""
import os

import pytest
import torch
import torch.nn as nn

from helpers import FP32_NORM_TOL, assert_parity
from oracle import dmpnn_ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _K():
    from notorch_amd import kernels

    return kernels


def _graph(kind="qm9", n=40, seed=0, rev_offset="nodes"):
    from notorch_amd.data.synth import make_batch

    return make_batch(kind, n, seed=seed).collate(rev_offset)


def _layout(G, rows):
    K = _K()
    dst_ptr, perm = K.csr_build(G.edge_index[1].contiguous().to(DEV), G.num_nodes)
    deg = (dst_ptr[1:] - dst_ptr[:-1]).cpu()
    maxdeg = int(deg.max())
    plan = K.tile_plan(dst_ptr, G.num_edges, maxdeg, rows=rows, ncu=K.PLAN_NCU)
    return perm, plan, maxdeg, bool((deg == 0).any())


def _ref_layer(G, H, S, W, b, residual, act, agg_act, reduce="sum"):
    src, dst, rev = G.edge_index[0], G.edge_index[1], G.rev_index
    A = S.double()[src] - act(H.double())[rev]
    U = nn.functional.linear(A, W.double(), None if b is None else b.double())
    Hn = H.double() + U if residual else U
    return Hn, dmpnn_ref.scatter(agg_act(Hn), dst, G.num_nodes, reduce)


@pytest.mark.parametrize("rev_offset", ["nodes", "edges"])
@pytest.mark.parametrize("h", [300, 256, 128, 36])
@pytest.mark.parametrize("exact_deg", [True, False])
def test_wide_plan_fused_layer(h, rev_offset, exact_deg):
    """Tiles of the kernel's capacity (plan balanced over the CUs); exact_deg passes the true max
    in-degree, else 32: same H_out, node sums bit-identical to the CPU scatter of the kernel's own
    H_out (the segmented scan sums each node's rows left to right)."""
    K = _K()
    G = _graph("qm9", 300, seed=h, rev_offset=rev_offset)
    E, V = G.num_edges, G.num_nodes
    g = torch.Generator().manual_seed(h + 1)
    H, S = torch.randn(E, h, generator=g), torch.randn(V, h, generator=g)
    lin = nn.Linear(h, h)
    W, b = lin.weight.detach(), lin.bias.detach()
    relu = K.act_code(nn.ReLU())
    cap = K.fused_tile_rows(h, torch.float32, relu, "sum", relu)
    assert cap == (64 if os.environ.get("NT_FK_NW") == "4" and h <= 320 else 128)  # NT_FK_NW=4: A/B walk
    perm, plan, maxdeg, zf = _layout(G, cap)
    assert max(int(x) for x in (plan[0][1:] - plan[0][:-1]).cpu()) <= cap
    amax_out = torch.zeros(2, device=DEV)
    Hn, Sn = K.dmpnn_update_fused(
        H.to(DEV), S.to(DEV), G.edge_index[0].to(DEV), G.rev_index.to(DEV), K.pack_weights(W.to(DEV)), b.to(DEV),
        residual=True, act=relu, plan=plan, tile_rows=cap, max_in_degree=maxdeg if exact_deg else 32, perm=perm,
        reduce="sum", agg_act=relu, zero_fill=zf, amax_out=amax_out,
    )
    rH, rS = _ref_layer(G, H, S, W, b, True, torch.relu, torch.relu)
    assert_parity(Hn, rH, FP32_NORM_TOL, f"H h={h}")
    assert_parity(Sn, rS, FP32_NORM_TOL, f"S h={h}")
    exact = dmpnn_ref.scatter(torch.relu(Hn.cpu()), G.edge_index[1], V, "sum")
    assert torch.equal(Sn.cpu(), exact)
    # amax_out = (max|H_out|, max|S_out|) exactly (the next layer's split scale)
    assert amax_out[0].item() == Hn.abs().max().item()
    assert amax_out[1].item() == Sn.abs().max().item()


@pytest.mark.parametrize("scale", [1e-6, 1e4, 3e7])
def test_split_scaling_far_from_unit_magnitude(scale):
    """Operands scaled by 1e-6 .. 3e7 (the fp16 parts would underflow / overflow unscaled): the
    amax-derived power-of-two scales keep the fp32 contract."""
    K = _K()
    h = 300
    G = _graph("qm9", 64, seed=3)
    E, V = G.num_edges, G.num_nodes
    g = torch.Generator().manual_seed(11)
    H, S = torch.randn(E, h, generator=g) * scale, torch.randn(V, h, generator=g) * scale
    W = torch.randn(h, h, generator=g) / h ** 0.5 * (1e-3 if scale > 1 else 1e3)
    perm, plan, maxdeg, zf = _layout(G, 64)
    relu = K.act_code(nn.ReLU())
    ident = K.act_code(nn.Identity())
    Hn, Sn = K.dmpnn_update_fused(
        H.to(DEV), S.to(DEV), G.edge_index[0].to(DEV), G.rev_index.to(DEV), K.pack_weights(W.to(DEV)), None,
        residual=True, act=relu, plan=plan, tile_rows=64, max_in_degree=maxdeg, perm=perm, reduce="sum",
        agg_act=ident, zero_fill=zf,
    )
    rH, rS = _ref_layer(G, H, S, W, None, True, torch.relu, lambda x: x)
    assert_parity(Hn, rH, FP32_NORM_TOL, f"H scale={scale}")
    assert_parity(Sn, rS, FP32_NORM_TOL, f"S scale={scale}")


@pytest.mark.parametrize("reduce", ["mean", "max", "min"])
def test_narrow_generic_reduce(reduce):
    """mean / max / min aggregation (the generic 64-row variant), node values bit-identical to the CPU
    scatter of the kernel's H_out."""
    K = _K()
    h = 300
    relu = K.act_code(nn.ReLU())
    assert K.fused_tile_rows(h, torch.float32, relu, reduce, relu) == 64
    assert K.fused_tile_rows(h, torch.float32, relu, "sum", relu) == 128
    G = _graph("qm9", 90, seed=7)
    E, V = G.num_edges, G.num_nodes
    g = torch.Generator().manual_seed(5)
    H, S = torch.randn(E, h, generator=g), torch.randn(V, h, generator=g)
    W = torch.randn(h, h, generator=g) / h ** 0.5
    perm, plan, maxdeg, zf = _layout(G, 64)
    Hn, Sn = K.dmpnn_update_fused(
        H.to(DEV), S.to(DEV), G.edge_index[0].to(DEV), G.rev_index.to(DEV), K.pack_weights(W.to(DEV)), None,
        residual=False, act=relu, plan=plan, tile_rows=64, max_in_degree=maxdeg, perm=perm, reduce=reduce,
        agg_act=relu, zero_fill=zf,
    )
    rH, _ = _ref_layer(G, H, S, W, None, False, torch.relu, torch.relu, reduce)
    assert_parity(Hn, rH, FP32_NORM_TOL, f"H {reduce}")
    exact = dmpnn_ref.scatter(torch.relu(Hn.cpu()), G.edge_index[1], V, reduce)
    assert torch.equal(Sn.cpu(), exact), reduce


def test_tile_capacity_is_checked():
    """A plan whose tiles exceed the kernel's capacity for the layer is refused (not truncated)."""
    K = _K()
    from notorch_amd._lib import NativeLibraryError

    h = 300
    G = _graph("qm9", 40, seed=2)
    E, V = G.num_edges, G.num_nodes
    perm, plan, maxdeg, zf = _layout(G, 128)
    relu = K.act_code(nn.ReLU())
    H, S = torch.randn(E, h, device=DEV), torch.randn(V, h, device=DEV)
    Wp = K.pack_weights(torch.randn(h, h, device=DEV))
    with pytest.raises(NativeLibraryError, match="tile plan rows"):
        K.dmpnn_update_fused(H, S, G.edge_index[0].to(DEV), G.rev_index.to(DEV), Wp, None, act=relu, plan=plan,
                             tile_rows=128, max_in_degree=maxdeg, perm=perm, reduce="max", agg_act=relu,
                             zero_fill=zf)


@pytest.mark.parametrize("h", [640, 1024])
@pytest.mark.parametrize("rev_offset", ["nodes", "edges"])
def test_block_wide_hidden(h, rev_offset):
    """ChempropBlock with hidden_dim > 512 (chemprop.py:54 takes any size): column-chunked fk kernel,
    fused aggregation, both rev modes, against the oracle."""
    from notorch_amd.nn import ChempropBlock, Sum

    G = _graph("qm9", 48, seed=h, rev_offset=rev_offset)
    torch.manual_seed(h)
    Xv, Xe = torch.randn(G.num_nodes, h), torch.randn(G.num_edges, h)
    blk = ChempropBlock(hidden_dim=h, depth=3).eval()
    Ws, bs = dmpnn_ref.block_params(blk)
    ref_n, ref_e = dmpnn_ref.chemprop_block(Xv, Xe, G.edge_index, G.rev_index, Ws, bs)
    ref_r = dmpnn_ref.readout(ref_n, G.batch_node_index, len(G), "sum")
    with torch.no_grad():
        out = blk.to(DEV)(G.update(node_feats=Xv, edge_feats=Xe).to(DEV))
        r = Sum()(out)
    assert_parity(out.edge_feats, ref_e, FP32_NORM_TOL, f"edge h={h}")
    assert_parity(out.node_feats, ref_n, FP32_NORM_TOL, f"node h={h}")
    assert_parity(r, ref_r, FP32_NORM_TOL, f"readout h={h}")


def test_block_wide_hidden_gradients():
    """Training at h = 640: kernel forward + kernel backward (fk dense dA, weight-grad kernel) against
    fp64 oracle autograd (smooth activation, no ReLU sign-flip floor)."""
    from notorch_amd.nn import ChempropBlock

    h = 640
    G = _graph("qm9", 16, seed=9)
    torch.manual_seed(1)
    Xv, Xe = torch.randn(G.num_nodes, h), torch.randn(G.num_edges, h)
    blk = ChempropBlock(hidden_dim=h, act=nn.SiLU, depth=2).train()
    Ws, bs = dmpnn_ref.block_params(blk)
    Xv64, Xe64 = Xv.double().requires_grad_(), Xe.double().requires_grad_()
    W64 = [w.double().requires_grad_() for w in Ws]
    b64 = [b.double().requires_grad_() for b in bs]
    n64, e64 = dmpnn_ref.chemprop_block(Xv64, Xe64, G.edge_index, G.rev_index, W64, b64, act=nn.SiLU())
    (n64.sum() + (e64 ** 2).mean()).backward()
    blk = blk.to(DEV)
    Xv_d, Xe_d = Xv.to(DEV).requires_grad_(), Xe.to(DEV).requires_grad_()
    out = blk(G.update(node_feats=Xv_d, edge_feats=Xe_d).to(DEV))
    (out.node_feats.sum() + (out.edge_feats ** 2).mean()).backward()
    assert_parity(Xv_d.grad, Xv64.grad, FP32_NORM_TOL, "dXv")
    assert_parity(Xe_d.grad, Xe64.grad, FP32_NORM_TOL, "dXe")
    for i, m in enumerate(blk._chemprop_layers()):
        assert_parity(m.linear.weight.grad, W64[i].grad, FP32_NORM_TOL, f"dW{i}")


def test_engine_uses_wide_plan_and_amax_chain():
    """The block at config-2 shape runs the 128-row plan (one launch per layer) and matches the
    oracle; the plan the collate shipped equals the device planner's."""
    from notorch_amd.nn import ChempropBlock
    from notorch_amd.nn.gnn import _engine

    K = _K()
    h = 300
    G = _graph("qm9", 512, seed=4)
    lay = G._nt_layout
    d_tp, d_n, _ = K.tile_plan(lay.dst_ptr.to(DEV), G.num_edges, lay.deg_range[0], rows=128, ncu=K.PLAN_NCU)
    assert d_n == lay.plan_wide[1] and torch.equal(d_tp.cpu(), lay.plan_wide[0])
    torch.manual_seed(0)
    Xv, Xe = torch.randn(G.num_nodes, h), torch.randn(G.num_edges, h)
    blk = ChempropBlock(hidden_dim=h, depth=3).eval()
    Ws, bs = dmpnn_ref.block_params(blk)
    ref_n, ref_e = dmpnn_ref.chemprop_block(Xv, Xe, G.edge_index, G.rev_index, Ws, bs)
    events = []
    _engine.UPDATE_EVENTS = events
    try:
        with torch.no_grad():
            out = blk.to(DEV)(G.update(node_feats=Xv, edge_feats=Xe).to(DEV))
    finally:
        _engine.UPDATE_EVENTS = None
    assert len(events) == 3 and _engine.LAST_UPDATE_INFO["kernel_short"] == "update_fk"
    assert_parity(out.edge_feats, ref_e, FP32_NORM_TOL, "edge")
    assert_parity(out.node_feats, ref_n, FP32_NORM_TOL, "node")


@pytest.mark.parametrize("h", [300, 36])
def test_plain_layer_without_aggregation(h):
    """No tile plan (the layerwise / hub path): fixed 64-row tiles in edge order, H_out only."""
    K = _K()
    G = _graph("qm9", 200, seed=h + 5)
    E, V = G.num_edges, G.num_nodes
    g = torch.Generator().manual_seed(h)
    H, S = torch.randn(E, h, generator=g), torch.randn(V, h, generator=g)
    lin = nn.Linear(h, h)
    W, b = lin.weight.detach(), lin.bias.detach()
    relu = K.act_code(nn.ReLU())
    Hn, Sn = K.dmpnn_update_fused(H.to(DEV), S.to(DEV), G.edge_index[0].to(DEV), G.rev_index.to(DEV),
                                  K.pack_weights(W.to(DEV)), b.to(DEV), residual=True, act=relu)
    assert Sn is None
    rH, _ = _ref_layer(G, H, S, W, b, True, torch.relu, torch.relu)
    assert_parity(Hn, rH, FP32_NORM_TOL, f"H h={h}")


@pytest.mark.parametrize("agg", ["relu", "identity", "tanh"])
def test_fused_aggregation_acts(agg):
    """Aggregation activations: relu / identity (fast variants) and a generic one (tanh)."""
    K = _K()
    h = 300
    acts = {"relu": (nn.ReLU(), torch.relu), "identity": (nn.Identity(), lambda x: x), "tanh": (nn.Tanh(), torch.tanh)}
    mod, fn = acts[agg]
    G = _graph("qm9", 120, seed=21)
    E, V = G.num_edges, G.num_nodes
    g = torch.Generator().manual_seed(21)
    H, S = torch.randn(E, h, generator=g), torch.randn(V, h, generator=g)
    W = torch.randn(h, h, generator=g) / h ** 0.5
    relu = K.act_code(nn.ReLU())
    perm, plan, maxdeg, zf = _layout(G, 64)
    Hn, Sn = K.dmpnn_update_fused(
        H.to(DEV), S.to(DEV), G.edge_index[0].to(DEV), G.rev_index.to(DEV), K.pack_weights(W.to(DEV)), None,
        residual=True, act=relu, plan=plan, tile_rows=64, max_in_degree=maxdeg, perm=perm, reduce="sum",
        agg_act=K.act_code(mod), zero_fill=zf,
    )
    rH, rS = _ref_layer(G, H, S, W, None, True, torch.relu, fn)
    assert_parity(Hn, rH, FP32_NORM_TOL, f"H {agg}")
    assert_parity(Sn, rS, FP32_NORM_TOL, f"S {agg}")
    if agg != "tanh":  # device tanh may differ from the CPU's by an ulp
        exact = dmpnn_ref.scatter(fn(Hn.cpu()), G.edge_index[1], V, "sum")
        assert torch.equal(Sn.cpu(), exact), agg


def test_pack_fk_only_matches_full_pack():
    """nt_dmpnn_pack_weight_fk writes the same fk image (scale header + fragments) as the full pack:
    dense_matmul on either image gives the same bits."""
    K = _K()
    g = torch.Generator().manual_seed(3)
    for h in (36, 300, 640):
        W = (torch.randn(h, h, generator=g) * 0.05).to(DEV)
        X = torch.randn(257, h, generator=g).to(DEV)
        full, fk = K.pack_weights(W), K.pack_weights(W, fk_only=True)
        a, b = K.dense_matmul(X, full), K.dense_matmul(X, fk)
        assert torch.equal(a, b), h
        assert_parity(a, X.double() @ W.double().t(), FP32_NORM_TOL, f"dense h={h}")


@pytest.mark.parametrize("h", [300, 36, 640])
def test_multi_pack_with_transposes_matches_single_packs(h):
    """nt_dmpnn_pack_weights_fk (all layers and their transposes in one launch pair, the training
    forward's pack) gives the bytes of the fk image of each W and of W.t().contiguous()."""
    K = _K()
    g = torch.Generator().manual_seed(h)
    Ws = [(torch.randn(h, h, generator=g) * 0.05).to(DEV) for _ in range(3)]
    imgs, imgsT = K.pack_weights_fk_multi(Ws, with_t=True)
    n = K.packed_weight_numel(h, torch.float32)
    for W, a, at in zip(Ws, imgs, imgsT):
        ref, refT = K.pack_weights(W, fk_only=True), K.pack_weights(W.t().contiguous(), fk_only=True)
        X = torch.randn(129, h, generator=g).to(DEV)
        assert torch.equal(K.dense_matmul(X, a), K.dense_matmul(X, ref)), h
        assert torch.equal(K.dense_matmul(X, at), K.dense_matmul(X, refT)), h
    only, none = K.pack_weights_fk_multi(Ws[:1])
    assert none is None and only[0].numel() == n


@pytest.mark.parametrize("h", [300, 128, 600])
@pytest.mark.parametrize("reduce", ["sum", "max"])
def test_fused_init_exact_on_skewed_degrees(h, reduce):
    """nt_dmpnn_init with the aggregation (the wave-per-node-chunk kernel, chemprop.py:82-83 fused with
    :37-39): a node of 150 in-edges (several 64-position index windows), runs of zero-in-degree nodes
    (inside and at the ends of a chunk), one or two column passes (h = 600).  H0 and S bit-identical to
    the CPU evaluation in the same order; amax raised to (max|H0|, max|S|) exactly."""
    K = _K()
    g = torch.Generator().manual_seed(h + len(reduce))
    V = 61
    deg = torch.randint(0, 6, (V,), generator=g)
    deg[0] = 150
    deg[3:6] = 0
    deg[8] = 0
    deg[-2:] = 0
    dst = torch.repeat_interleave(torch.arange(V), deg)
    dst = dst[torch.randperm(dst.numel(), generator=g)]
    E = dst.numel()
    src = torch.randint(0, V, (E,), generator=g)
    Xv, Xe = torch.randn(V, h, generator=g), torch.randn(E, h, generator=g)
    dst_ptr, perm = K.csr_build(dst.to(DEV), V)
    relu = K.act_code(nn.ReLU())
    am = torch.zeros(2, device=DEV)
    H0, S = K.dmpnn_init(Xv.to(DEV), Xe.to(DEV), src.to(DEV), dst_ptr, perm, act=relu, reduce=reduce, amax=am)
    rH = Xv[src] + Xe
    assert torch.equal(H0.cpu(), rH)
    rS = dmpnn_ref.scatter(torch.relu(rH), dst, V, reduce)
    assert torch.equal(S.cpu(), rS)
    assert am[0].item() == rH.abs().max().item()
    assert am[1].item() == rS.abs().max().item()
    am.zero_()
    H0b, none = K.dmpnn_init(Xv.to(DEV), Xe.to(DEV), src.to(DEV), amax=am)  # no aggregation: S entry untouched
    assert none is None and torch.equal(H0b.cpu(), rH)
    assert am[0].item() == rH.abs().max().item() and am[1].item() == 0.0


def test_amax_ring_wraps_bitexact():
    """Forwards that keep no states take their split-scale rows from a per-stream ring that is zeroed
    once per wrap (_engine._amax_buffer): 2.5 wraps of no-grad forwards give bit-identical outputs."""
    from notorch_amd.nn import ChempropBlock, Sum
    from notorch_amd.nn.gnn import _engine

    G = _graph("qm9", 64, seed=5)
    h = 128
    g = torch.Generator().manual_seed(6)
    Gd = G.update(node_feats=torch.randn(G.num_nodes, h, generator=g),
                  edge_feats=torch.randn(G.num_edges, h, generator=g)).to(DEV)
    blk = ChempropBlock(hidden_dim=h, depth=3).to(DEV).eval()
    with torch.no_grad():
        first = Sum()(blk(Gd))
        outs = [Sum()(blk(Gd)) for _ in range(int(2.5 * _engine._AMAX_RING))]
    torch.cuda.synchronize()
    assert all(torch.equal(first, o) for o in outs)
    key = next(k for k in _engine._amax_rings if k[2] == 3)
    assert _engine._amax_rings[key][0].shape == (_engine._AMAX_RING, 4, 2)
