"""GPU: hub nodes (in-degree > 32, polymer graphs, BASELINE config 5) on the fused fp32 layer.

The tile plan cuts hubs at the stride (nt_dmpnn_tile_plan_hubs), the fused kernel leaves the hubs'
aggregation out (row table marked by nt_dmpnn_mark_hub_rows) and nt_dmpnn_hub_aggregate adds it
(chemprop.py:37-39, :86 with torch_scatter semantics).  Checked against the oracle at 1e-5.
"""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from helpers import assert_parity
from oracle import dmpnn_ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _polymer(n, seed, rev_offset="nodes"):
    from notorch_amd.data.synth import make_batch

    return make_batch("polymer", n, seed=seed).collate(rev_offset)


def test_device_hub_plans_match_host():
    """The device planners (hub info, nt_dmpnn_tile_plan_hubs) give the collate's host plans."""
    from notorch_amd import kernels as K
    from notorch_amd.data.models.graph import DeviceLayout
    from notorch_amd.nn.gnn import _engine

    P = _polymer(3, seed=7)
    lay = P._nt_layout
    ids, nhub, rest = lay.hubs
    assert nhub > 0 and rest <= _engine.HUB_DEGREE
    for rows, (tile_ptr, ntiles) in ((64, lay.plan[:2]), (128, lay.plan_wide)):
        tp, n, dsts = K.tile_plan(lay.dst_ptr.to(DEV), P.num_edges, rest, rows=rows, ncu=K.PLAN_NCU,
                                  hub_degree=_engine.HUB_DEGREE)
        assert n == ntiles and torch.equal(tp.cpu(), tile_ptr)
        assert torch.equal(dsts.cpu(), lay.plan[2])
    d = DeviceLayout(lay.dst_ptr.to(DEV), lay.dst_perm.to(DEV))
    hub = _engine.hub_info(d)
    assert torch.equal(hub[0].cpu(), ids) and hub[1:] == (nhub, rest)
    # the base row table carries every row's node; the hub sub-run table (hub_run_table) turns exactly
    # the hubs' rows into sub-runs of <= max_in_degree rows inside one tile, slots in dst order
    rt0 = _engine.row_table(d, dsts, P.edge_index[0].to(DEV), P.rev_index.to(DEV), P.num_nodes)
    assert (rt0[:, 3] >= 0).all()
    tile_ptr = lay.plan_wide[0].to(DEV)
    rt, nslots, hubs, slot_ptr = _engine.hub_run_table(d, rt0, tile_ptr, dsts, rest)
    rt = rt.cpu()
    is_hub = torch.zeros(P.num_nodes, dtype=torch.bool)
    is_hub[ids.long()] = True
    hub_row = is_hub[lay.plan[2].long()]
    w = rt[:, 3]
    assert torch.equal(w < 0, hub_row) and torch.equal(hubs.cpu(), ids)
    wv = -w[hub_row] - 1
    slot, fl = wv >> 2, wv & 3
    starts = torch.nonzero(fl & 1).flatten()
    ends = torch.nonzero(fl & 2).flatten()
    assert starts.numel() == ends.numel() == nslots and torch.equal(slot[starts], torch.arange(nslots))
    assert ((ends - starts + 1) <= rest).all() and ((ends - starts) >= 0).all()
    sp = slot_ptr.cpu().long()
    assert int(sp[-1]) == nslots and int(sp[0]) == 0 and (sp[ids.long() + 1] > sp[ids.long()]).all()


_ACTS = {"relu": (nn.ReLU(), torch.relu), "identity": (nn.Identity(), lambda x: x), "silu": (nn.SiLU(), F.silu)}


@pytest.mark.parametrize("reduce", ["sum", "mean", "max", "min"])
@pytest.mark.parametrize("act", ["relu", "identity", "silu"])
def test_hub_aggregate_matches_scatter(reduce, act):
    """nt_dmpnn_hub_aggregate writes the hub rows only, torch_scatter's reduce of act(X) over their
    in-edges, and raises amax to their max |value|."""
    from notorch_amd import kernels as K

    P = _polymer(2, seed=3, rev_offset="edges")
    lay = P._nt_layout
    ids = lay.hubs[0]
    E, V, h = P.num_edges, P.num_nodes, 300
    X = torch.randn(E, h, generator=torch.Generator().manual_seed(1))
    mod, fn = _ACTS[act]
    out = torch.full((V, h), 7.0, device=DEV)
    amax = torch.zeros(1, device=DEV)
    K.hub_aggregate(X.to(DEV), lay.dst_perm.to(DEV), lay.dst_ptr.to(DEV), ids.to(DEV), out, reduce=reduce,
                    act=K.act_code(mod), amax=amax)
    ref = dmpnn_ref.scatter(fn(X.double()), P.edge_index[1], V, reduce)
    o = out.cpu()
    hub = ids.long()
    assert_parity(o[hub], ref[hub], what=f"hubs {reduce} {act}")
    rest = torch.ones(V, dtype=torch.bool)
    rest[hub] = False
    assert (o[rest] == 7.0).all()
    assert amax.item() == o[hub].abs().max().item()


@pytest.mark.parametrize("reduce,act,residual", [("sum", nn.ReLU, True), ("mean", nn.ReLU, True),
                                                 ("max", nn.ReLU, False), ("sum", nn.SiLU, True)])
def test_block_on_hubs_runs_fused(reduce, act, residual):
    """A polymer block takes the fused path (d + 1 layer launches + one hub launch per layer) and
    matches the oracle: 128-row plan for relu / sum, 64-row plan otherwise."""
    from notorch_amd.nn import ChempropBlock
    from notorch_amd.nn.gnn import _engine

    G = _polymer(2, seed=11)
    h = 64
    torch.manual_seed(0)
    Xv, Xe = torch.randn(G.num_nodes, h), torch.randn(G.num_edges, h)
    blk = ChempropBlock(hidden_dim=h, depth=3, act=act, reduce=reduce, residual=residual).eval()
    Ws, bs = dmpnn_ref.block_params(blk)
    ref_n, ref_e = dmpnn_ref.chemprop_block(Xv, Xe, G.edge_index, G.rev_index, Ws, bs, act=act(),
                                            residual=residual, reduce=reduce)
    with torch.no_grad():
        out = blk.to(DEV)(G.update(node_feats=Xv, edge_feats=Xe).to(DEV))
    assert _engine.LAST_UPDATE_INFO["fused"]
    assert_parity(out.edge_feats, ref_e, what="edge")
    assert_parity(out.node_feats, ref_n, what="node")


def test_hub_block_deterministic_and_grads():
    """Two forwards are bit-identical; training through the fused hub forward matches the oracle's
    autograd (fp64)."""
    from notorch_amd.nn import ChempropBlock, Sum

    G = _polymer(2, seed=5)
    ei, rev, bni, B = G.edge_index.clone(), G.rev_index.clone(), G.batch_node_index.clone(), len(G)
    h = 32
    torch.manual_seed(1)
    Xv, Xe = torch.randn(G.num_nodes, h), torch.randn(G.num_edges, h)
    blk = ChempropBlock(hidden_dim=h, depth=2, act=nn.SiLU).to(DEV)  # smooth: no relu'(0) ties
    xv, xe = Xv.to(DEV).requires_grad_(), Xe.to(DEV).requires_grad_()
    Gd = G.to(DEV).update(node_feats=xv, edge_feats=xe)
    with torch.no_grad():
        a = blk(Gd).node_feats.clone()
        b = blk(Gd).node_feats.clone()
    assert torch.equal(a, b)
    out = Sum()(blk(Gd))
    out.square().sum().backward()
    Ws, bs = dmpnn_ref.block_params(blk)
    Xv64, Xe64 = Xv.double().requires_grad_(), Xe.double().requires_grad_()
    W64 = [w.double().requires_grad_() for w in Ws]
    b64 = [x.double().requires_grad_() for x in bs]
    rn, _ = dmpnn_ref.chemprop_block(Xv64, Xe64, ei, rev, W64, b64, act=F.silu)
    dmpnn_ref.readout(rn, bni, B, "sum").square().sum().backward()
    lin0 = blk.layers[0].module.update[0]
    assert_parity(xv.grad, Xv64.grad, 1e-4, "dXv")
    assert_parity(xe.grad, Xe64.grad, 1e-4, "dXe")
    assert_parity(lin0.weight.grad, W64[0].grad, 1e-4, "dW0")


def test_amax_outputs_of_the_producers():
    """The kernels that write an fp32 operand of the fp16-split kernels report its max |value|
    exactly (ABI 3): the plain init (H0), the chunked reduce (S of hub graphs), the backward's row
    gather and edge backward (G)."""
    from notorch_amd import kernels as K
    from notorch_amd.nn.gnn import _engine

    G = _polymer(2, seed=4)
    lay = G._nt_layout
    E, V, h = G.num_edges, G.num_nodes, 64
    g = torch.Generator().manual_seed(0)
    Xv, Xe = torch.randn(V, h, generator=g).to(DEV), torch.randn(E, h, generator=g).to(DEV) * 3
    src, dst = G.edge_index[0].to(DEV), G.edge_index[1].to(DEV)
    dst_ptr, perm = lay.dst_ptr.to(DEV), lay.dst_perm.to(DEV)
    am = torch.zeros(2, device=DEV)
    H0, _ = K.dmpnn_init(Xv, Xe, src, amax=am)
    assert am[0].item() == H0.abs().max().item()
    chunks = K.chunk_plan(dst_ptr)
    S = K.segment_reduce_chunked(H0, dst_ptr, perm, V, chunks, act=K.act_code(nn.ReLU()), amax=am[1:2])
    assert am[1].item() == S.abs().max().item()
    dnode = torch.randn(V, h, generator=g).to(DEV)
    gm = torch.zeros(1, device=DEV)
    Gr = K.gather_rows(dnode, dst, base=H0, amax=gm)
    assert gm.item() == Gr.abs().max().item()
    rev = G.rev_index.to(DEV)
    rev_ptr, rev_perm = K.csr_build(rev, E, check_bounds=False)
    dA = torch.randn(E, h, generator=g).to(DEV)
    dS = torch.randn(V, h, generator=g).to(DEV)
    gm2 = torch.zeros(1, device=DEV)
    Gn = K.dmpnn_edge_backward(Gr, H0, dA, dS, dst, rev_ptr, rev_perm, dst_ptr, amax=gm2)
    assert gm2.item() == Gn.abs().max().item()
    assert _engine.hub_info(lay) is not None


@pytest.mark.parametrize("reduce", ["sum", "mean", "max"])
def test_fused_chunked_init_matches_init_then_chunked_reduce(reduce):
    """nt_dmpnn_init_chunked (hub graphs, fp32): H0 bit-identical to nt_dmpnn_init, S bit-identical to
    nt_segment_reduce_chunked of that H0 (same chunks, same order), amax exact; h = 300 (16-B pieces)
    and h = 30 (scalar pieces)."""
    from notorch_amd import kernels as K

    G = _polymer(2, seed=7)
    lay = G._nt_layout
    E, V = G.num_edges, G.num_nodes
    src = G.edge_index[0].to(DEV)
    dst_ptr, perm = lay.dst_ptr.to(DEV), lay.dst_perm.to(DEV)
    chunks = K.chunk_plan(dst_ptr)
    relu = K.act_code(nn.ReLU())
    for h in (300, 30):
        g = torch.Generator().manual_seed(h)
        Xv, Xe = torch.randn(V, h, generator=g).to(DEV), torch.randn(E, h, generator=g).to(DEV)
        am = torch.zeros(2, device=DEV)
        H0, S = K.dmpnn_init_chunked(Xv, Xe, src, dst_ptr, perm, chunks, act=relu, reduce=reduce, amax=am)
        rH, _ = K.dmpnn_init(Xv, Xe, src)
        rS = K.segment_reduce_chunked(rH, dst_ptr, perm, V, chunks, reduce=reduce, act=relu)
        assert torch.equal(H0, rH)
        assert torch.equal(S, rS)
        assert am[0].item() == rH.abs().max().item() and am[1].item() == rS.abs().max().item()


def test_padded_rows_chunked_init_and_hub_aggregate_bit_identical():
    """ABI 7 row pitches on the hub-graph path: nt_dmpnn_init_chunked's ld_out and
    nt_dmpnn_hub_aggregate's ld give the dense-row values bit for bit."""
    from notorch_amd import kernels as K
    from notorch_amd.data.synth import make_batch

    G = make_batch("polymer", 2, seed=4).collate("nodes").to(DEV)
    lay = G._nt_layout
    V, E, h = G.num_nodes, G.num_edges, 300
    torch.manual_seed(0)
    Xv, Xe = torch.randn(V, h, device=DEV), torch.randn(E, h, device=DEV)
    src = G.edge_index[0].contiguous()
    chunks = K.chunk_plan(lay.dst_ptr)
    relu = K.act_code(nn.ReLU())
    deg = lay.dst_ptr[1:] - lay.dst_ptr[:-1]
    hubs = torch.nonzero(deg > 32).flatten().to(torch.int32)
    res = {}
    for ld in (h, 304):
        am = torch.zeros(2, device=DEV)
        H0, S = K.dmpnn_init_chunked(Xv, Xe, src, lay.dst_ptr, lay.dst_perm, chunks, act=relu, amax=am, pitch=ld)
        assert H0.stride(0) == ld and S.stride(0) == ld
        out = K.padded_rows(V, h, ld, torch.float32, DEV)
        out.zero_()
        K.hub_aggregate(H0, lay.dst_perm, lay.dst_ptr, hubs, out, act=relu)
        res[ld] = (H0.contiguous(), S.contiguous(), am, out.contiguous())
    for name, a, b in zip(("H0", "S", "amax", "hub out"), res[h], res[304]):
        assert torch.equal(a, b), name


@pytest.mark.parametrize("rows", [64, 128])
@pytest.mark.parametrize("reduce", ["sum", "mean", "max"])
def test_hub_subrun_partials_and_combine(rows, reduce):
    """ABI 7 hub partials: with the row table's hub rows cut into sub-runs (kernels.hub_runs: within a
    tile, at most max_in_degree rows), the fused layer writes each sub-run's reduce as a partial row and
    hub_combine finishes the hubs' S_out rows; every node row against the oracle scatter of the layer
    output, the non-hub rows bit-identical to the plain fused run's."""
    from notorch_amd import kernels as K
    from notorch_amd.data.synth import make_batch
    from notorch_amd.nn.gnn import _engine

    G = make_batch("polymer", 2, seed=8).collate("nodes").to(DEV)
    lay = G._nt_layout
    V, E, h = G.num_nodes, G.num_edges, 64
    torch.manual_seed(1)
    H, S = torch.randn(E, h, device=DEV), torch.randn(V, h, device=DEV)
    W, b = torch.randn(h, h, device=DEV) / 8, torch.randn(h, device=DEV)
    Wp = K.pack_weights(W)
    src, rev = G.edge_index[0].contiguous(), G.rev_index
    relu = K.act_code(nn.ReLU())
    rows = min(rows, K.fused_tile_rows(h, torch.float32, relu, reduce, relu))
    plan = _engine.fused_plan(lay, V, E, rows)
    tile_ptr, ntiles, dsts, zf = plan
    maxdeg = _engine.fused_max_in_degree(lay)
    rt0 = K.dmpnn_row_table(lay.dst_perm, dsts, src, rev, V)
    rt, nslots, hubs, slot_ptr = K.hub_runs(rt0, lay.dst_ptr, dsts, tile_ptr, _engine.HUB_DEGREE, maxdeg)
    assert nslots > 0 and int(slot_ptr[-1]) == nslots
    w = rt[:, 3]
    assert (w < 0).sum() > 0 and torch.equal(rt[:, :3], rt0[:, :3])
    part = torch.empty(nslots, h, device=DEV)
    am = torch.zeros(2, 2, device=DEV)
    K.absmax(H, am[0, 0:1])
    K.absmax(S, am[0, 1:2])
    out, Sn = K.dmpnn_update_fused(H, S, src, rev, Wp, b, act=relu, plan=(tile_ptr, ntiles, dsts), tile_rows=rows,
                                   max_in_degree=maxdeg, perm=lay.dst_perm, reduce=reduce, agg_act=relu,
                                   zero_fill=True, amax_in=am[0], row_table=rt, S_part=part)
    K.hub_combine(part, hubs, slot_ptr, lay.dst_ptr, Sn, reduce=reduce)
    ref = dmpnn_ref.scatter(torch.relu(out.cpu()), G.edge_index[1].cpu(), V, reduce)
    assert_parity(Sn, ref, 1e-5, f"S_out with hub partials ({reduce})")
    if reduce == "max":
        assert torch.equal(Sn.cpu(), ref)


def test_split_hub_init_bit_identical_to_chunked_init():
    """Hub graphs' init (round 5): the wave-per-node init skipping nodes of in-degree > 32 (ABI 7
    skip_degree) plus the chunked init over the hubs' chunks alone (chunk_ids) give the full chunked
    init's H0, S and amax bit for bit."""
    from notorch_amd import kernels as K
    from notorch_amd.data.synth import make_batch
    from notorch_amd.nn.gnn import _engine

    G = make_batch("polymer", 3, seed=9).collate("nodes").to(DEV)
    lay = G._nt_layout
    V, E, h = G.num_nodes, G.num_edges, 300
    torch.manual_seed(4)
    Xv, Xe = torch.randn(V, h, device=DEV), torch.randn(E, h, device=DEV)
    src = G.edge_index[0].contiguous()
    relu = K.act_code(nn.ReLU())
    chunks = _engine.dst_chunks(lay)
    assert chunks is not None
    am0, am1 = torch.zeros(2, device=DEV), torch.zeros(2, device=DEV)
    H_ref, S_ref = K.dmpnn_init_chunked(Xv, Xe, src, lay.dst_ptr, lay.dst_perm, chunks, act=relu, amax=am0,
                                        pitch=304)
    H, S = K.dmpnn_init(Xv, Xe, src, lay.dst_ptr, lay.dst_perm, act=relu, amax=am1, pitch=304,
                        skip_degree=_engine.MAX_FUSED_IN_DEGREE)
    ids = _engine.hub_chunk_ids(lay, chunks)
    assert 0 < ids.numel() < chunks[1]
    K.dmpnn_init_chunked(Xv, Xe, src, lay.dst_ptr, lay.dst_perm, chunks, act=relu, amax=am1, pitch=304, H0=H, S=S,
                         chunk_ids=ids)
    assert torch.equal(H, H_ref) and torch.equal(S, S_ref) and torch.equal(am0, am1)
