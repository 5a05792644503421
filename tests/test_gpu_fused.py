"""GPU parity of the persistent fused layer kernel (nt_dmpnn_update_fused) and its tile plan.

The kernel computes one layer (chemprop.py:36-43, residual.py:27-28) and, with a tile plan, the
aggregation the next layer consumes (chemprop.py:37-39) or the final node scatter (chemprop.py:86).
Reference: the fp64 restatement of the same ops; criterion FP32_NORM_TOL; the tile
plan and the node sums' order are checked exactly.
"""
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


def _csr(G):
    K = _K()
    return K.csr_build(G.edge_index[1].contiguous().to(DEV), G.num_nodes)


def _plan(G):
    K = _K()
    dst_ptr, perm = _csr(G)
    deg = (dst_ptr[1:] - dst_ptr[:-1]).cpu()
    tile_ptr, ntiles, dsts = K.tile_plan(dst_ptr, G.num_edges, int(deg.max()))
    return dst_ptr, perm, (tile_ptr, ntiles, dsts), bool((deg == 0).any())


def test_tile_plan_invariants():
    G = _graph("qm9", 300, seed=5)
    dst_ptr, perm, (tile_ptr, ntiles, dsts), _ = _plan(G)
    tp = tile_ptr.cpu().long()
    dp = dst_ptr.cpu().long()
    E = G.num_edges
    assert tp[0] == 0 and tp[-1] == E and len(tp) == ntiles + 1
    sizes = tp[1:] - tp[:-1]
    assert (sizes > 0).all() and (sizes <= 64).all()
    # every cut is a node boundary of the dst CSR
    assert torch.isin(tp, dp).all()
    # dst_sorted[p] == dst of the edge at position p
    dst = G.edge_index[1]
    assert torch.equal(dsts.cpu().long(), dst[perm.cpu().long()])


def _ref_layer(G, H, S, W, b, residual, act, reduce, agg_act):
    src, dst, rev = G.edge_index[0], G.edge_index[1], G.rev_index
    Hd, Sd = H.double(), S.double()
    A = Sd[src] - act(Hd)[rev]
    U = nn.functional.linear(A, W.double(), None if b is None else b.double())
    Hn = Hd + U if residual else U
    Sn = dmpnn_ref.scatter(agg_act(Hn), dst, G.num_nodes, reduce)
    return Hn, Sn


@pytest.mark.parametrize("h", [300, 296, 256, 100, 36])
@pytest.mark.parametrize("rev_offset", ["nodes", "edges"])
def test_fused_layer(h, rev_offset):
    K = _K()
    G = _graph("qm9", 45, seed=h, rev_offset=rev_offset)
    E, V = G.num_edges, G.num_nodes
    g = torch.Generator().manual_seed(h)
    H, S = torch.randn(E, h, generator=g), torch.randn(V, h, generator=g)
    lin = nn.Linear(h, h)
    W, b = lin.weight.detach(), lin.bias.detach()
    _, perm, plan, zf = _plan(G)
    Wp = K.pack_weights(W.to(DEV))
    relu = K.act_code(nn.ReLU())
    Hn, Sn = K.dmpnn_update_fused(
        H.to(DEV), S.to(DEV), G.edge_index[0].to(DEV), G.rev_index.to(DEV), Wp, b.to(DEV),
        residual=True, act=relu, plan=plan, perm=perm, reduce="sum", agg_act=relu, zero_fill=zf,
    )
    rH, rS = _ref_layer(G, H, S, W, b, True, torch.relu, "sum", torch.relu)
    assert_parity(Hn, rH, FP32_NORM_TOL, f"H h={h}")
    assert_parity(Sn, rS, FP32_NORM_TOL, f"S h={h}")
    # the node sums are exactly the CPU scatter_add_ of the kernel's own H_out (ascending edge id)
    exact = dmpnn_ref.scatter(torch.relu(Hn.cpu()), G.edge_index[1], V, "sum")
    assert torch.equal(Sn.cpu(), exact)


@pytest.mark.parametrize("reduce", ["sum", "mean", "max", "min"])
@pytest.mark.parametrize("agg", ["relu", "identity"])
def test_fused_reduce_and_final_scatter(reduce, agg):
    K = _K()
    h = 64
    G = _graph("qm9", 30, seed=11)
    E, V = G.num_edges, G.num_nodes
    g = torch.Generator().manual_seed(3)
    H, S = torch.randn(E, h, generator=g), torch.randn(V, h, generator=g)
    W = torch.randn(h, h, generator=g) / 8
    _, perm, plan, zf = _plan(G)
    act_mod = nn.ReLU() if agg == "relu" else nn.Identity()
    Hn, Sn = K.dmpnn_update_fused(
        H.to(DEV), S.to(DEV), G.edge_index[0].to(DEV), G.rev_index.to(DEV), K.pack_weights(W.to(DEV)),
        None, residual=False, act=K.act_code(nn.ReLU()), plan=plan, perm=perm, reduce=reduce,
        agg_act=K.act_code(act_mod), zero_fill=zf,
    )
    rH, rS = _ref_layer(G, H, S, W, None, False, torch.relu, reduce, act_mod)
    assert_parity(Hn, rH, FP32_NORM_TOL, "H")
    exact = dmpnn_ref.scatter(act_mod(Hn.cpu()), G.edge_index[1], V, reduce)
    assert torch.equal(Sn.cpu(), exact), reduce


def test_fused_runtime_activation():
    K = _K()
    h = 100
    G = _graph("qm9", 20, seed=2)
    E, V = G.num_edges, G.num_nodes
    g = torch.Generator().manual_seed(9)
    H, S = torch.randn(E, h, generator=g), torch.randn(V, h, generator=g)
    W = torch.randn(h, h, generator=g) / 10
    _, perm, plan, zf = _plan(G)
    for act in (nn.SiLU(), nn.Tanh(), nn.ELU()):
        code = K.act_code(act)
        Hn, Sn = K.dmpnn_update_fused(
            H.to(DEV), S.to(DEV), G.edge_index[0].to(DEV), G.rev_index.to(DEV),
            K.pack_weights(W.to(DEV)), None, residual=True, act=code, plan=plan, perm=perm,
            agg_act=code, zero_fill=zf,
        )
        rH, rS = _ref_layer(G, H, S, W, None, True, act, "sum", act)
        assert_parity(Hn, rH, FP32_NORM_TOL, type(act).__name__)
        assert_parity(Sn, rS, FP32_NORM_TOL, type(act).__name__)


def test_unfused_persistent_matches_update():
    """plan=None: the persistent kernel computes exactly nt_dmpnn_update's H_out."""
    K = _K()
    h = 300
    G = _graph("qm9", 70, seed=4)
    E, V = G.num_edges, G.num_nodes
    g = torch.Generator().manual_seed(1)
    H, S = torch.randn(E, h, generator=g).to(DEV), torch.randn(V, h, generator=g).to(DEV)
    lin = nn.Linear(h, h).to(DEV)
    Wp = K.pack_weights(lin.weight.detach())
    src, rev = G.edge_index[0].to(DEV), G.rev_index.to(DEV)
    relu = K.act_code(nn.ReLU())
    Hn, Sn = K.dmpnn_update_fused(H, S, src, rev, Wp, lin.bias.detach(), residual=True, act=relu)
    assert Sn is None
    with torch.no_grad():
        ref = H.double() + nn.functional.linear(
            S.double()[src] - torch.relu(H.double())[rev], lin.weight.double(), lin.bias.double()
        )
    assert_parity(Hn, ref, FP32_NORM_TOL, "unfused persistent")


def test_fused_zero_in_degree_nodes():
    """A node without in-edges gets S_out = 0 (torch_scatter's empty segment), via zero_fill."""
    from notorch_amd.data.models.graph import BatchedGraph, Graph

    K = _K()
    h = 32
    gs = [
        Graph(torch.zeros(3, 7, dtype=torch.long), torch.zeros(4, 2, dtype=torch.long),
              torch.tensor([[0, 1, 1, 2], [1, 0, 2, 1]]), torch.tensor([1, 0, 3, 2])),
        Graph(torch.zeros(1, 7, dtype=torch.long), torch.zeros(0, 2, dtype=torch.long),
              torch.zeros(2, 0, dtype=torch.long), torch.zeros(0, dtype=torch.long)),
        Graph(torch.zeros(2, 7, dtype=torch.long), torch.zeros(2, 2, dtype=torch.long),
              torch.tensor([[0, 1], [1, 0]]), torch.tensor([1, 0])),
    ]
    G = BatchedGraph.from_graphs(gs, rev_offset="edges")
    E, V = G.num_edges, G.num_nodes
    g = torch.Generator().manual_seed(0)
    H, S = torch.randn(E, h, generator=g), torch.randn(V, h, generator=g)
    W = torch.randn(h, h, generator=g) / 5
    _, perm, plan, zf = _plan(G)
    assert zf
    relu = K.act_code(nn.ReLU())
    Hn, Sn = K.dmpnn_update_fused(
        H.to(DEV), S.to(DEV), G.edge_index[0].to(DEV), G.rev_index.to(DEV), K.pack_weights(W.to(DEV)),
        None, residual=True, act=relu, plan=plan, perm=perm, agg_act=relu, zero_fill=zf,
    )
    rH, rS = _ref_layer(G, H, S, W, None, True, torch.relu, "sum", torch.relu)
    assert_parity(Hn, rH, FP32_NORM_TOL, "H")
    assert_parity(Sn, rS, FP32_NORM_TOL, "S")
    assert (Sn[3] == 0).all()


@pytest.mark.parametrize("fused", ["1", "0"])
def test_block_paths_agree(fused, monkeypatch):
    """ChempropBlock through the fused path and through the unfused path, against the oracle."""
    from notorch_amd.nn import ChempropBlock

    monkeypatch.setenv("NT_FUSED", fused)
    h = 300
    G = _graph("qm9", 64, seed=8)
    torch.manual_seed(0)
    Xv, Xe = torch.randn(G.num_nodes, h), torch.randn(G.num_edges, h)
    blk = ChempropBlock(hidden_dim=h, depth=3).eval()
    Ws, bs = dmpnn_ref.block_params(blk)
    ref_node, ref_edge = dmpnn_ref.chemprop_block(Xv, Xe, G.edge_index, G.rev_index, Ws, bs)
    Gd = G.update(node_feats=Xv, edge_feats=Xe).to(DEV)
    with torch.no_grad():
        out = blk.to(DEV)(Gd)
    assert_parity(out.edge_feats, ref_edge, FP32_NORM_TOL, f"edge fused={fused}")
    assert_parity(out.node_feats, ref_node, FP32_NORM_TOL, f"node fused={fused}")


@pytest.mark.parametrize("variant", ["pk", "ps"])
def test_fused_kernel_variants_and_no_spin_timeouts(variant, monkeypatch):
    """Both persistent kernels (NT_FUSED_KERNEL) agree with the oracle; the pk ring's bounded spins
    never gave up (nt_debug_pk_timeouts)."""
    import ctypes

    from notorch_amd import _lib

    K = _K()
    if not _lib.DIAG:
        pytest.skip("the pk / ps ring kernels are A/B variants: diagnostic library only (NT_LIB=diag)")
    monkeypatch.setenv("NT_FUSED_KERNEL", variant)
    lib = _lib.load()
    fn = lib.nt_debug_pk_timeouts
    fn.argtypes = [ctypes.POINTER(ctypes.c_uint), ctypes.c_int]
    cnt = ctypes.c_uint(0)
    assert fn(ctypes.byref(cnt), 1) == 0
    for h, n, rev_offset in ((300, 300, "nodes"), (300, 7, "edges"), (100, 50, "nodes"), (32, 20, "nodes")):
        G = _graph("qm9", n, seed=h + n, rev_offset=rev_offset)
        E, V = G.num_edges, G.num_nodes
        g = torch.Generator().manual_seed(n)
        H, S = torch.randn(E, h, generator=g), torch.randn(V, h, generator=g)
        lin = nn.Linear(h, h)
        W, b = lin.weight.detach(), lin.bias.detach()
        _, perm, plan, zf = _plan(G)
        relu = K.act_code(nn.ReLU())
        args = (H.to(DEV), S.to(DEV), G.edge_index[0].to(DEV), G.rev_index.to(DEV),
                K.pack_weights(W.to(DEV)), b.to(DEV))
        Hn, Sn = K.dmpnn_update_fused(*args, residual=True, act=relu, plan=plan, perm=perm,
                                      agg_act=relu, zero_fill=zf)
        rH, rS = _ref_layer(G, H, S, W, b, True, torch.relu, "sum", torch.relu)
        assert_parity(Hn, rH, FP32_NORM_TOL, f"{variant} H h={h} n={n}")
        assert_parity(Sn, rS, FP32_NORM_TOL, f"{variant} S h={h} n={n}")
        Hu, _ = K.dmpnn_update_fused(*args, residual=True, act=relu)
        assert_parity(Hu, rH, FP32_NORM_TOL, f"{variant} unfused H h={h} n={n}")
    torch.cuda.synchronize()
    assert fn(ctypes.byref(cnt), 1) == 0
    assert cnt.value == 0, "a pk ring spin gave up"


def test_host_plans_equal_device_planners():
    """The collate's host tile / chunk plans are the arrays nt_dmpnn_tile_plan and
    kernels.chunk_plan build on the device (the engine uses them without a sync)."""
    from notorch_amd.data.synth import make_batch

    K = _K()
    for kind, n in (("qm9", 500), ("zinc", 64)):
        G = make_batch(kind, n, seed=3).collate("nodes")
        lay = G._nt_layout
        tile_ptr, ntiles, dsts, _ = lay.plan
        d_tile_ptr, d_ntiles, d_dsts = K.tile_plan(lay.dst_ptr.to(DEV), G.num_edges, lay.deg_range[0], rows=64,
                                                   ncu=K.PLAN_SLOTS64)
        assert d_ntiles == ntiles
        assert torch.equal(d_tile_ptr.cpu(), tile_ptr) and torch.equal(d_dsts.cpu(), dsts)
    P = make_batch("polymer", 2, seed=2).collate("nodes")
    lay = P._nt_layout
    for host, seg_ptr in ((lay.dst_chunks, lay.dst_ptr), (lay.mol_chunks[1], lay.mol_ptr)):
        dev = K.chunk_plan(seg_ptr.to(DEV))
        assert dev[1] == host[1]
        assert torch.equal(dev[0].cpu(), host[0]) and torch.equal(dev[2].cpu(), host[2])
        assert torch.equal(dev[3].cpu(), host[3]) and torch.equal(dev[4].cpu(), host[4])


def test_forward_on_a_non_current_device():
    """Every launch runs under a device guard (kernels._run): a block on cuda:1 while cuda:0 is
    current gives the same result as on cuda:0 (skipped on one-GPU boxes)."""
    from notorch_amd.nn import ChempropBlock

    if torch.cuda.device_count() < 2:
        pytest.skip("needs two visible GPUs")
    G = _graph("qm9", 64, seed=12)
    h = 300
    torch.manual_seed(0)
    Xv, Xe = torch.randn(G.num_nodes, h), torch.randn(G.num_edges, h)
    blk = ChempropBlock(hidden_dim=h, depth=3).eval()
    outs = []
    for dev in ("cuda:0", "cuda:1"):
        with torch.cuda.device(0), torch.no_grad():
            b = blk.to(dev)
            outs.append(b(G.update(node_feats=Xv, edge_feats=Xe).to(dev)).edge_feats.cpu())
    assert torch.equal(outs[0], outs[1])


def _n_for_tiles(pred, lo, hi, step=1):
    """Smallest molecule count in [lo, hi) whose fused tile plan's ntiles satisfies pred."""
    for n in range(lo, hi, step):
        _, _, (_, ntiles, _), _ = _plan(_graph("qm9", n, seed=11))
        if pred(ntiles):
            return n, ntiles
    pytest.skip("no batch size in range gives the wanted tile count")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", ["grid_eq_ntiles_mult8", "ragged_over_cus"])
def test_xcd_walk_branches(dtype, case):
    """Both branches of the XCD-aware tile walk (update_pk.hip / bf16.hip): (a) grid == ntiles with
    ntiles % 8 == 0 (one tile per block, XCD chunks of ntiles / 8), (b) more tiles than resident
    blocks with ntiles % 8 != 0 (ragged per-XCD chunks, several tiles per block)."""
    K = _K()
    slots = torch.cuda.get_device_properties(0).multi_processor_count * (2 if dtype == torch.bfloat16 else 1)
    if case == "grid_eq_ntiles_mult8":
        n, ntiles = _n_for_tiles(lambda t: t % 8 == 0 and 16 <= t <= slots, 20, 400)
    else:
        n, ntiles = _n_for_tiles(lambda t: t % 8 != 0 and t > slots + 3, 4 * slots, 8 * slots, 7)
    G = _graph("qm9", n, seed=11)
    h = 64
    g = torch.Generator().manual_seed(n)
    H, S = torch.randn(G.num_edges, h, generator=g), torch.randn(G.num_nodes, h, generator=g)
    lin = nn.Linear(h, h)
    W, b = lin.weight.detach(), lin.bias.detach()
    if dtype == torch.bfloat16:
        H, S, W, b = (x.to(torch.bfloat16).float() for x in (H, S, W, b))
    _, perm, plan, zf = _plan(G)
    relu = K.act_code(nn.ReLU())
    Hn, Sn = K.dmpnn_update_fused(H.to(dtype).to(DEV), S.to(dtype).to(DEV), G.edge_index[0].to(DEV),
                                  G.rev_index.to(DEV), K.pack_weights(W.to(dtype).to(DEV)),
                                  b.to(dtype).to(DEV), residual=True, act=relu, plan=plan, perm=perm,
                                  agg_act=relu, zero_fill=zf)
    rH, rS = _ref_layer(G, H, S, W, b, True, torch.relu, "sum", torch.relu)
    tol = FP32_NORM_TOL if dtype == torch.float32 else 2e-2
    assert_parity(Hn.float(), rH, tol, f"{case} H ntiles={ntiles}")
    assert_parity(Sn.float(), rS, tol, f"{case} S ntiles={ntiles}")


@pytest.mark.parametrize("kernel", ["fk", "pk"])
@pytest.mark.parametrize("h,M", [(300, 77_000), (300, 1), (100, 1000), (64, 4097), (4, 3)])
def test_dense_matmul(h, M, kernel):
    """nt_dmpnn_dense_matmul (the backward's dA = G W, chemprop.py:41 under autograd): the fp16x3 fk
    kernel's and the bf16x6 pk kernel's dense modes against fp64, fp32 contract."""
    K = _K()
    g = torch.Generator().manual_seed(M + h)
    X, W = torch.randn(M, h, generator=g), torch.randn(h, h, generator=g) / h ** 0.5
    out = K.dense_matmul(X.to(DEV), K.pack_weights(W.t().contiguous().to(DEV)), kernel=kernel)
    ref = X.double() @ W.double()
    assert_parity(out, ref, FP32_NORM_TOL, f"dense {kernel} h={h} M={M}")


@pytest.mark.parametrize("h,M", [(640, 3000), (1024, 700)])
def test_dense_matmul_wide_hidden(h, M):
    """Hidden sizes beyond 512 (the reference takes any hidden_dim, chemprop.py:54): the fk kernel's
    column chunks in dense mode."""
    K = _K()
    g = torch.Generator().manual_seed(M + h)
    X, W = torch.randn(M, h, generator=g), torch.randn(h, h, generator=g) / h ** 0.5
    out = K.dense_matmul(X.to(DEV), K.pack_weights(W.t().contiguous().to(DEV)))
    assert_parity(out, X.double() @ W.double(), FP32_NORM_TOL, f"dense h={h} M={M}")


@pytest.mark.parametrize("h,E,act", [(300, 77_840, "relu"), (300, 1, "relu"), (100, 1000, "identity"),
                                     (64, 4097, "gelu"), (4, 3, "relu"), (512, 3000, "tanh"),
                                     (300, 33, "leaky_relu")])
def test_weight_grad_x6(h, E, act):
    """nt_dmpnn_weight_grad (the backward's dW = G^T A and db = colsum G of nn.Linear at
    chemprop.py:26,41, A = S[src] - act(H[rev]) of chemprop.py:40 formed in the kernel) against fp64,
    fp32 contract; also bit-identical on a repeat (fixed-order split-K reduction)."""
    K = _K()
    mods = {"relu": nn.ReLU(), "identity": nn.Identity(), "gelu": nn.GELU(), "tanh": nn.Tanh(),
            "leaky_relu": nn.LeakyReLU(0.1)}
    mod = mods[act]
    g = torch.Generator().manual_seed(E + h)
    V = max(E // 2, 1)
    Gr, H, S = torch.randn(E, h, generator=g), torch.randn(E, h, generator=g), torch.randn(V, h, generator=g)
    src = torch.randint(0, V, (E,), generator=g)
    rev = torch.randint(0, E, (E,), generator=g)
    dW, db = K.weight_grad(Gr.to(DEV), H.to(DEV), S.to(DEV), src.to(DEV), rev.to(DEV), act=K.act_code(mod))
    A = S.double()[src] - mod(H.double())[rev]
    assert_parity(dW, Gr.double().t() @ A, FP32_NORM_TOL, f"dW h={h} E={E} {act}")
    assert_parity(db, Gr.double().sum(0), FP32_NORM_TOL, f"db h={h} E={E}")
    dW2, db2 = K.weight_grad(Gr.to(DEV), H.to(DEV), S.to(DEV), src.to(DEV), rev.to(DEV), act=K.act_code(mod))
    assert torch.equal(dW, dW2) and torch.equal(db, db2)
    # dense mode (no gathers): dW = G^T S
    dWd, _ = K.weight_grad(Gr.to(DEV), None, H.to(DEV), None, None, bias=False)
    assert_parity(dWd, Gr.double().t() @ H.double(), FP32_NORM_TOL, f"dense dW h={h} E={E}")


def test_weight_grad_no_edges():
    K = _K()
    Z = torch.empty(0, 16, device=DEV)
    dW, db = K.weight_grad(Z, Z, torch.randn(3, 16, device=DEV), torch.empty(0, dtype=torch.long, device=DEV),
                           torch.empty(0, dtype=torch.long, device=DEV))
    assert torch.count_nonzero(dW) == 0 and torch.count_nonzero(db) == 0


@pytest.mark.parametrize("h,E,act,gs,xs", [(300, 77_840, "relu", 1.0, 1.0), (300, 1, "relu", 1.0, 1.0),
                                            (100, 1000, "identity", 1e-6, 1e3), (64, 4097, "gelu", 1e4, 1e-3),
                                            (4, 3, "relu", 1.0, 1.0), (320, 5000, "tanh", 1.0, 1.0),
                                            (300, 33, "leaky_relu", 3.0, 0.5), (36, 20_000, "silu", 1e-20, 1e10)])
def test_weight_grad_fk(h, E, act, gs, xs):
    """nt_dmpnn_weight_grad_fk (two-part fp16 split on the forward's bounds) against fp64 at the fp32
    contract, over magnitudes that need the power-of-two scales (G from 1e-20 to 1e4, H / S from 1e-3
    to 1e10) and with bounds above the true maxima (any bound >= max works); bit-identical repeat."""
    K = _K()
    mods = {"relu": nn.ReLU(), "identity": nn.Identity(), "gelu": nn.GELU(), "tanh": nn.Tanh(),
            "leaky_relu": nn.LeakyReLU(0.1), "silu": nn.SiLU()}
    mod = mods[act]
    g = torch.Generator().manual_seed(E + h + 1)
    V = max(E // 2, 1)
    Gr = torch.randn(E, h, generator=g) * gs
    H, S = torch.randn(E, h, generator=g) * xs, torch.randn(V, h, generator=g) * xs
    src = torch.randint(0, V, (E,), generator=g)
    rev = torch.randint(0, E, (E,), generator=g)
    amax_G = torch.tensor([Gr.abs().max().item() * 1.7], device=DEV)
    amax_HS = torch.tensor([H.abs().max().item(), S.abs().max().item() * 1.3], device=DEV)
    args = (Gr.to(DEV), H.to(DEV), S.to(DEV), src.to(DEV), rev.to(DEV))
    dW, db = K.weight_grad(*args, act=K.act_code(mod), amax_G=amax_G, amax_HS=amax_HS)
    A = S.double()[src] - mod(H.double())[rev]
    assert_parity(dW, Gr.double().t() @ A, FP32_NORM_TOL, f"dW h={h} E={E} {act}")
    assert_parity(db, Gr.double().sum(0), FP32_NORM_TOL, f"db h={h} E={E}")
    dW2, db2 = K.weight_grad(*args, act=K.act_code(mod), amax_G=amax_G, amax_HS=amax_HS)
    assert torch.equal(dW, dW2) and torch.equal(db, db2)


@pytest.mark.parametrize("h,pitch", [(300, 304), (300, 320), (132, 136)])
@pytest.mark.parametrize("rows", [64, 128])
def test_row_padded_init_and_layer_bit_identical(h, pitch, rows):
    """Row-padded H / S (ABI 7 ld_out of nt_dmpnn_init, ld_in / ld_out of nt_dmpnn_update_fused):
    the same values, bit for bit, as the dense rows -- the pitch moves rows, not arithmetic -- for a
    padded -> padded layer and a padded -> dense one (the block's last layer)."""
    K = _K()
    G = _graph("qm9", 200, seed=21)
    V, E = G.num_nodes, G.num_edges
    dst_ptr, perm, plan, zf = _plan(G)
    deg = int((dst_ptr[1:] - dst_ptr[:-1]).max())
    plan = K.tile_plan(dst_ptr, E, deg, rows=rows, ncu=K.PLAN_NCU)
    torch.manual_seed(3)
    Xv, Xe = torch.randn(V, h, device=DEV), torch.randn(E, h, device=DEV)
    W, b = torch.randn(h, h, device=DEV) / h ** 0.5, torch.randn(h, device=DEV)
    Wp = K.pack_weights(W)
    src, rev = G.edge_index[0].contiguous().to(DEV), G.rev_index.to(DEV)
    relu = K.act_code(nn.ReLU())
    ident = K.act_code(nn.Identity())
    outs = {}
    for ld in (h, pitch):
        am = torch.zeros(3, 2, device=DEV)
        H0, S0 = K.dmpnn_init(Xv, Xe, src, dst_ptr, perm, act=relu, amax=am[0], pitch=ld)
        assert H0.shape == (E, h) and H0.stride(0) == ld and S0.stride(0) == ld
        rt = K.dmpnn_row_table(perm, plan[2], src, rev, V)
        H1, S1 = K.dmpnn_update_fused(H0, S0, src, rev, Wp, b, act=relu, plan=plan, tile_rows=rows,
                                      max_in_degree=deg, perm=perm, agg_act=relu, zero_fill=zf, amax_in=am[0],
                                      amax_out=am[1], row_table=rt, pitch_out=ld)
        assert H1.stride(0) == ld and S1.stride(0) == ld
        H2, S2 = K.dmpnn_update_fused(H1, S1, src, rev, Wp, b, act=relu, plan=plan, tile_rows=rows,
                                      max_in_degree=deg, perm=perm, agg_act=ident, zero_fill=zf, amax_in=am[1],
                                      amax_out=am[2], row_table=rt)
        assert H2.is_contiguous() and S2.is_contiguous()
        outs[ld] = [t.contiguous() for t in (H0, S0, H1, S1, H2, S2)] + [am]
    for name, a, c in zip(("H0", "S0", "H1", "S1", "H2", "S2", "amax"), outs[h], outs[pitch]):
        assert torch.equal(a, c), name


@pytest.mark.parametrize("kind,n", [("qm9", 300), ("polymer", 2)])
def test_block_forward_row_padding_is_invisible(monkeypatch, kind, n):
    """The inference forward runs its intermediate layers on row-padded buffers (h = 300 -> 304, or
    320 on hub graphs; hub graphs too: the chunked init, the hub aggregation): the block's outputs are dense tensors and
    equal, bit for bit, to the dense-row forward."""
    from notorch_amd.nn import ChempropBlock
    from notorch_amd.nn.gnn import _engine

    G = _graph(kind, n, seed=22)
    h = 300
    torch.manual_seed(5)
    Xv, Xe = torch.randn(G.num_nodes, h), torch.randn(G.num_edges, h)
    blk = ChempropBlock(hidden_dim=h, depth=3).to(DEV).eval()
    Gd = G.update(node_feats=Xv, edge_feats=Xe).to(DEV)
    res = {}
    for pad, align in ((True, 8), (True, 32), (False, 0)):  # 304 (32-B sectors), 320 (128-B lines), dense
        monkeypatch.setattr(_engine, "_ROW_PAD", pad)
        monkeypatch.setattr(_engine, "_ROW_ALIGN", align)
        with torch.no_grad():
            out = blk(Gd)
        assert out.node_feats.is_contiguous() and out.edge_feats.is_contiguous()
        res[(pad, align)] = (out.node_feats.clone(), out.edge_feats.clone())
    monkeypatch.setattr(_engine, "_ROW_PAD", True)
    monkeypatch.setattr(_engine, "_ROW_ALIGN", 32)
    assert _engine.row_pitch(h, torch.float32) == 320
    monkeypatch.setattr(_engine, "_ROW_ALIGN", 8)
    assert _engine.row_pitch(h, torch.float32) == 304
    for key in ((True, 8), (True, 32)):
        assert torch.equal(res[key][0], res[(False, 0)][0]) and torch.equal(res[key][1], res[(False, 0)][1])
