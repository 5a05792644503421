"""GPU parity: the HIP kernels (through the C ABI) against the CPU oracle on identical inputs.

Criterion: fp32 normalised max error max|gpu - ref| / max|ref| <= 1e-5; integer
outputs (CSR) bit-exact; properties (batching invariance in fixed-rev mode, determinism) bit-exact.
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

from helpers import FP32_NORM_TOL, assert_parity, chain3, diatomic, load_golden
from oracle import dmpnn_ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _K():
    from notorch_amd import kernels

    return kernels


def _graph_tensors(kind="qm9", n=32, seed=0, rev_offset="nodes"):
    from notorch_amd.data.synth import make_batch

    return make_batch(kind, n, seed=seed).collate(rev_offset)


def _embed(G, h, seed=0):
    torch.manual_seed(seed)
    nt = nn.EmbeddingBag(42, h, mode="sum")
    et = nn.EmbeddingBag(13, h, mode="sum")
    with torch.no_grad():
        return nt(G.node_feats), et(G.edge_feats)


# ------------------------------------------------------------------ native library is what runs
def test_native_library_loaded():
    from notorch_amd import _lib

    lib = _lib.load()
    assert lib.nt_abi_version() == _lib.ABI_VERSION


# ------------------------------------------------------------------ CSR (bit-exact)
@pytest.mark.parametrize("n,nseg", [(0, 5), (1, 1), (1000, 37), (77840, 36408), (200_000, 3)])
def test_csr_build_exact(n, nseg):
    K = _K()
    g = torch.Generator().manual_seed(n + nseg)
    idx = torch.randint(0, max(nseg, 1), (n,), generator=g) if nseg else torch.zeros(0, dtype=torch.long)
    seg_ptr, perm = K.csr_build(idx.to(DEV), nseg)
    exp_perm = np.argsort(idx.numpy(), kind="stable")
    exp_ptr = np.concatenate([[0], np.cumsum(np.bincount(idx.numpy(), minlength=nseg))])
    assert np.array_equal(seg_ptr.cpu().numpy(), exp_ptr)
    assert np.array_equal(perm.cpu().numpy(), exp_perm)


def test_csr_build_out_of_range_raises():
    K = _K()
    idx = torch.tensor([0, 3, 1], device=DEV)
    with pytest.raises(IndexError):
        K.csr_build(idx, 3)


# ------------------------------------------------------------------ segment reduce
@pytest.mark.parametrize("reduce", ["sum", "mean", "max", "min"])
@pytest.mark.parametrize("h", [300, 13])
@pytest.mark.parametrize("act", [nn.Identity(), nn.ReLU(), nn.GELU(), nn.LeakyReLU(0.1)])
def test_segment_reduce(reduce, h, act):
    K = _K()
    G = _graph_tensors("qm9", 64, seed=1)
    E, V = G.edge_index.shape[1], G.num_nodes
    X = torch.randn(E, h)
    dst = G.edge_index[1]
    seg_ptr, perm = K.csr_build(dst.to(DEV), V)
    out = K.segment_reduce(X.to(DEV), seg_ptr, perm, V, reduce=reduce, act=K.act_code(act))
    ref = dmpnn_ref.scatter(act(X), dst, V, reduce)
    assert_parity(out, ref, 1e-6, f"segment_reduce {reduce}")
    if reduce == "sum" and isinstance(act, nn.Identity):
        # ascending-edge-order accumulation == CPU scatter_add_: bit-exact
        assert torch.equal(out.cpu(), ref)


@pytest.mark.parametrize("reduce", ["sum", "mean", "max", "min"])
@pytest.mark.parametrize("h", [300, 13])
def test_dmpnn_aggregate(reduce, h):
    """nt_dmpnn_aggregate (SURVEY §8(b)'s name): the layer's relu + scatter (chemprop.py:36-39)."""
    K = _K()
    G = _graph_tensors("qm9", 64, seed=2)
    E, V = G.edge_index.shape[1], G.num_nodes
    X = torch.randn(E, h)
    dst = G.edge_index[1]
    seg_ptr, perm = K.csr_build(dst.to(DEV), V)
    out = K.dmpnn_aggregate(X.to(DEV), seg_ptr, perm, V, reduce=reduce)
    ref = dmpnn_ref.scatter(torch.relu(X), dst, V, reduce)
    assert_parity(out, ref, 1e-6, f"dmpnn_aggregate {reduce}")
    if reduce in ("sum", "max", "min"):  # ascending-edge-order accumulation: bit-exact
        assert torch.equal(out.cpu(), ref)


@pytest.mark.parametrize("h", [128, 200, 300, 320, 336])
@pytest.mark.parametrize("reduce", ["sum", "mean", "max", "min"])
def test_segment_reduce_contiguous_segments(h, reduce):
    """perm = None (the readouts' node rows, stored molecule by molecule): segments of 0..27 rows, so
    the block kernel's 10-row chunks, ragged last chunks and empty segments are all hit; h 128..320
    takes segment_reduce_block, 336 the row-piece kernel.  Sum is the CPU scatter_add_ order: bit-exact;
    max / min / empty bit-exact too."""
    K = _K()
    g = torch.Generator().manual_seed(h)
    sizes = torch.randint(0, 28, (300,), generator=g)
    sizes[::17] = 0
    idx = torch.repeat_interleave(torch.arange(len(sizes)), sizes)
    X = torch.randn(len(idx), h, generator=g)
    seg_ptr = torch.zeros(len(sizes) + 1, dtype=torch.int32)
    seg_ptr[1:] = torch.cumsum(sizes, 0)
    out = K.segment_reduce(X.to(DEV), seg_ptr.to(DEV), None, len(sizes), reduce=reduce)
    ref = dmpnn_ref.scatter(X, idx, len(sizes), reduce)
    assert_parity(out, ref, 1e-6, f"contiguous segment_reduce {reduce} h={h}")
    if reduce != "mean":
        assert torch.equal(out.cpu(), ref)


def test_segment_reduce_empty_segments():
    K = _K()
    X = torch.randn(3, 8)
    idx = torch.tensor([4, 4, 1])  # segments 0, 2, 3, 5 are empty
    seg_ptr, perm = K.csr_build(idx.to(DEV), 6)
    for red in ("sum", "mean", "max", "min"):
        out = K.segment_reduce(X.to(DEV), seg_ptr, perm, 6, reduce=red)
        assert torch.equal(out.cpu(), dmpnn_ref.scatter(X, idx, 6, red)), red


# ------------------------------------------------------------------ fused layer update
@pytest.mark.parametrize("h", [300, 256, 64, 100, 13, 2, 512])
@pytest.mark.parametrize("residual", [True, False])
def test_update_kernel(h, residual):
    K = _K()
    G = _graph_tensors("qm9", 48, seed=h)
    E, V = G.edge_index.shape[1], G.num_nodes
    g = torch.Generator().manual_seed(h)
    H = torch.randn(E, h, generator=g)
    S = torch.randn(V, h, generator=g)
    lin = nn.Linear(h, h)
    src, rev = G.edge_index[0], G.rev_index
    out = K.dmpnn_update(
        H.to(DEV), S.to(DEV), src.to(DEV), rev.to(DEV), K.pack_weights(lin.weight.detach().to(DEV)),
        lin.bias.detach().to(DEV), residual=residual, act=K.act_code(nn.ReLU()),
    )
    with torch.no_grad():
        A = S.double()[src] - torch.relu(H.double())[rev]
        ref = nn.functional.linear(A, lin.weight.double(), lin.bias.double())
        if residual:
            ref = H.double() + ref
    assert_parity(out, ref, FP32_NORM_TOL, f"update h={h}")


@pytest.mark.parametrize("variant", ["as", "x6", "ring", "tile"])
@pytest.mark.parametrize("h", [300, 296, 256, 100, 36])
def test_update_kernel_variants(variant, h, monkeypatch):
    """Every selectable update kernel (NT_UPDATE_KERNEL) of the diagnostic library against the fp64
    restatement.  The shipping library ignores NT_UPDATE_KERNEL (one fixed dispatch, covered by
    test_update_kernel), so these run only under NT_LIB=diag."""
    from notorch_amd import _lib

    if not _lib.DIAG:
        pytest.skip("kernel variants are selectable only in the diagnostic library (NT_LIB=diag)")
    K = _K()
    monkeypatch.setenv("NT_UPDATE_KERNEL", variant)
    G = _graph_tensors("qm9", 37, seed=h + 1)
    E, V = G.edge_index.shape[1], G.num_nodes
    g = torch.Generator().manual_seed(h + 7)
    H = torch.randn(E, h, generator=g)
    S = torch.randn(V, h, generator=g)
    lin = nn.Linear(h, h)
    src, rev = G.edge_index[0], G.rev_index
    out = K.dmpnn_update(
        H.to(DEV), S.to(DEV), src.to(DEV), rev.to(DEV), K.pack_weights(lin.weight.detach().to(DEV)),
        lin.bias.detach().to(DEV), residual=True, act=K.act_code(nn.ReLU()),
    )
    with torch.no_grad():
        A = S.double()[src] - torch.relu(H.double())[rev]
        ref = H.double() + nn.functional.linear(A, lin.weight.double(), lin.bias.double())
    assert_parity(out, ref, FP32_NORM_TOL, f"update[{variant}] h={h}")


def test_update_kernel_no_bias_and_acts():
    K = _K()
    G = _graph_tensors("qm9", 16, seed=3)
    E, V, h = G.edge_index.shape[1], G.num_nodes, 64
    H, S = torch.randn(E, h), torch.randn(V, h)
    W = torch.randn(h, h) / 8
    src, rev = G.edge_index[0], G.rev_index
    for act in (nn.Identity(), nn.SiLU(), nn.Tanh(), nn.ELU(), nn.Sigmoid()):
        out = K.dmpnn_update(
            H.to(DEV), S.to(DEV), src.to(DEV), rev.to(DEV), K.pack_weights(W.to(DEV)), None,
            residual=True, act=K.act_code(act),
        )
        ref = H + nn.functional.linear(S[src] - act(H)[rev], W)
        assert_parity(out, ref, FP32_NORM_TOL, type(act).__name__)


# ------------------------------------------------------------------ module-level parity
def _module_forward(G, Xv, Xe, Ws, bs, **kw):
    from notorch_amd.nn import ChempropBlock

    h = Xv.shape[1]
    blk = ChempropBlock(hidden_dim=h, depth=len(Ws), **kw).to(DEV).eval()
    with torch.no_grad():
        for m, W, b in zip(blk._chemprop_layers(), Ws, bs):
            m.linear.weight.copy_(W)
            if b is not None:
                m.linear.bias.copy_(b)
    Gd = G.update(node_feats=Xv, edge_feats=Xe).to(DEV)
    with torch.no_grad():
        return blk, Gd, blk(Gd)


def test_kat_chain3_on_device():
    from notorch_amd.data.models.graph import BatchedGraph

    Xv, Xe, ei, rev, W, b, H1, node = chain3()
    G = BatchedGraph(Xv, Xe, ei, rev, batch_node_index=torch.zeros(3, dtype=torch.long),
                     batch_edge_index=torch.zeros(4, dtype=torch.long), size=1)
    _, _, out = _module_forward(G, Xv, Xe, [W], [b])
    assert torch.equal(out.edge_feats.cpu(), H1)
    assert torch.equal(out.node_feats.cpu(), node)


def test_kat_diatomic_on_device():
    from notorch_amd.data.models.graph import Graph

    Xv, Xe, ei, rev, Ws, bs = diatomic(h=300, depth=3)
    G = Graph(Xv, Xe, ei, rev)
    _, _, out = _module_forward(G, Xv, Xe, Ws, bs)
    H = Xv[ei[0]] + Xe
    for b in bs:
        H = H + b
    assert torch.equal(out.edge_feats.cpu(), H)
    assert torch.equal(out.node_feats.cpu(), H[[1, 0]])


@pytest.mark.parametrize("name", ["tiny.npz", "config1.npz"])
def test_golden_fixture(name):
    from notorch_amd.data.models.graph import BatchedGraph
    from notorch_amd.nn import Sum

    z = load_golden(name)
    t = {k: torch.from_numpy(v) for k, v in z.items()}
    G = BatchedGraph(t["node_feats"], t["edge_feats"], t["edge_index"], t["rev_index"],
                     batch_node_index=t["batch_node_index"], batch_edge_index=t["batch_edge_index"],
                     size=int(z["size"]))
    _, Gd, out = _module_forward(G, t["node_feats"], t["edge_feats"], list(t["W"]), list(t["b"]))
    assert_parity(out.edge_feats, t["out_edge"], what="edge_feats")
    assert_parity(out.node_feats, t["out_node"], what="node_feats")
    with torch.no_grad():
        r = Sum()(out)
    assert_parity(r, t["out_sum"], what="readout")
    assert_parity(r, t["out_sum64"], what="readout vs fp64")


@pytest.mark.parametrize(
    "opts",
    [
        dict(),
        dict(shared=True),
        dict(residual=False),
        dict(bias=False),
        dict(reduce="mean"),
        dict(reduce="max"),
        dict(reduce="min"),
        dict(act=nn.LeakyReLU),
        dict(act=nn.GELU),
    ],
    ids=lambda o: ",".join(f"{k}={getattr(v, '__name__', v)}" for k, v in o.items()) or "default",
)
def test_block_options(opts):
    G = _graph_tensors("qm9", 40, seed=7)
    h, depth = 96, 3
    Xv, Xe = _embed(G, h, seed=1)
    from notorch_amd.nn import ChempropBlock

    torch.manual_seed(5)
    blk = ChempropBlock(hidden_dim=h, depth=depth, **opts).eval()
    Ws, bs = dmpnn_ref.block_params(blk)
    act = blk._chemprop_layers()[0].act
    ref_n, ref_e = dmpnn_ref.chemprop_block(
        Xv, Xe, G.edge_index, G.rev_index, Ws, bs, act=act, residual=opts.get("residual", True),
        reduce=opts.get("reduce", "sum"),
    )
    blk = blk.to(DEV)
    with torch.no_grad():
        out = blk(G.update(node_feats=Xv, edge_feats=Xe).to(DEV))
    assert_parity(out.edge_feats, ref_e, what="edge")
    assert_parity(out.node_feats, ref_n, what="node")


@pytest.mark.parametrize("depth", [0, 1, 5])
def test_block_depths(depth):
    G = _graph_tensors("zinc", 24, seed=depth)
    Xv, Xe = _embed(G, 64)
    torch.manual_seed(0)
    Ws = [torch.randn(64, 64) / 8 for _ in range(depth)]
    bs = [torch.randn(64) for _ in range(depth)]
    ref_n, ref_e = dmpnn_ref.chemprop_block(Xv, Xe, G.edge_index, G.rev_index, Ws, bs)
    _, _, out = _module_forward(G, Xv, Xe, Ws, bs)
    assert_parity(out.edge_feats, ref_e, what="edge")
    assert_parity(out.node_feats, ref_n, what="node")


@pytest.mark.parametrize("reduce,cls", [("sum", "Sum"), ("mean", "Mean"), ("max", "Max"), ("min", "Min")])
def test_readouts(reduce, cls):
    import notorch_amd.nn as ntnn

    G = _graph_tensors("qm9", 50, seed=11)
    X = torch.randn(G.num_nodes, 300)
    Gd = G.update(node_feats=X).to(DEV)
    out = getattr(ntnn, cls)()(Gd)
    ref = dmpnn_ref.readout(X, G.batch_node_index, len(G), reduce)
    assert torch.equal(out.cpu(), ref) or reduce in ("mean",)
    assert_parity(out, ref, 1e-6, cls)


def test_readout_unsorted_batch_index():
    from notorch_amd.data.models.graph import BatchedGraph
    from notorch_amd.nn import Sum

    G = _graph_tensors("qm9", 8, seed=2)
    p = torch.randperm(G.num_nodes)
    X = torch.randn(G.num_nodes, 32)
    bni = G.batch_node_index[p]
    BG = BatchedGraph(X, G.edge_feats, G.edge_index, G.rev_index, batch_node_index=bni,
                      batch_edge_index=G.batch_edge_index, size=8).to(DEV)
    out = Sum()(BG)
    assert_parity(out, dmpnn_ref.readout(X, bni, 8, "sum"), 1e-6, "unsorted")


# ------------------------------------------------------------------ full-size configs
def test_config2_qm9_4096_parity():
    """BASELINE config 2 shape: 4096 QM9-shaped molecules, h=300, depth=3, fp32, vs the oracle."""
    G = _graph_tensors("qm9", 4096, seed=0)
    h = 300
    Xv, Xe = _embed(G, h, seed=0)
    torch.manual_seed(1)
    Ws = [nn.Linear(h, h).weight.detach() for _ in range(3)]
    bs = [torch.randn(h) * 0.05 for _ in range(3)]
    torch.set_num_threads(min(16, torch.get_num_threads()))
    ref_n, ref_e = dmpnn_ref.chemprop_block(Xv, Xe, G.edge_index, G.rev_index, Ws, bs)
    ref_r = dmpnn_ref.readout(ref_n, G.batch_node_index, len(G), "sum")
    from notorch_amd.nn import Sum

    _, _, out = _module_forward(G, Xv, Xe, Ws, bs)
    with torch.no_grad():
        r = Sum()(out)
    assert_parity(out.edge_feats, ref_e, what="edge")
    assert_parity(out.node_feats, ref_n, what="node")
    assert_parity(r, ref_r, what="readout")


def test_polymer_hubs_parity():
    """Config 5 shape (reduced to 4 graphs): 1k-10k atoms, hub in-degree up to ~512."""
    G = _graph_tensors("polymer", 4, seed=5, rev_offset="edges")
    h = 128
    Xv, Xe = _embed(G, h, seed=2)
    torch.manual_seed(3)
    Ws = [torch.randn(h, h) / 16 for _ in range(3)]
    bs = [torch.randn(h) * 0.1 for _ in range(3)]
    ref_n, ref_e = dmpnn_ref.chemprop_block(Xv, Xe, G.edge_index, G.rev_index, Ws, bs)
    _, _, out = _module_forward(G, Xv, Xe, Ws, bs)
    assert_parity(out.edge_feats, ref_e, what="edge")
    assert_parity(out.node_feats, ref_n, what="node")


@pytest.mark.parametrize("rev_offset", ["nodes", "edges"])
def test_polymer_bench_config_parity(rev_offset):
    """BASELINE config 5 exactly as bench.py runs it (16 polymer graphs of 1k-10k atoms, hubs of
    in-degree up to ~512, seed 1000, h = 300, depth 3, default init), in the reference collate's
    compat rev mode and in fixed mode: block outputs and the Sum readout against the oracle
    (chemprop.py:81-88 with the scatter over hub segments at :39 / :86, agg.py:23-29)."""
    from notorch_amd.data.synth import make_batch
    from notorch_amd.nn import ChempropBlock, Sum

    G = make_batch("polymer", 16, seed=1000).collate(rev_offset)
    assert G.num_nodes > 40_000 and int(torch.bincount(G.edge_index[1]).max()) >= 100
    h = 300
    Xv, Xe = _embed(G, h, seed=0)
    torch.manual_seed(0)
    blk = ChempropBlock(hidden_dim=h, depth=3).eval()
    Ws, bs = dmpnn_ref.block_params(blk)
    ref_n, ref_e = dmpnn_ref.chemprop_block(Xv, Xe, G.edge_index, G.rev_index, Ws, bs)
    ref_r = dmpnn_ref.readout(ref_n, G.batch_node_index, len(G), "sum")
    Gd = G.update(node_feats=Xv, edge_feats=Xe).to(DEV)
    with torch.no_grad():
        out = blk.to(DEV)(Gd)
        r = Sum()(out)
    assert_parity(out.edge_feats, ref_e, what=f"edge {rev_offset}")
    assert_parity(out.node_feats, ref_n, what=f"node {rev_offset}")
    assert_parity(r, ref_r, what=f"readout {rev_offset}")


def test_fixed_mode_batching_invariance_bitexact():
    """Fixed-rev collate: forward(batch) == concat(forward(shard_i)) bit for bit, at full size."""
    from notorch_amd.data.synth import make_batch

    batch = make_batch("qm9", 4096, seed=9)
    h = 300
    torch.manual_seed(0)
    Ws = [torch.randn(h, h) / 17 for _ in range(3)]
    bs = [torch.randn(h) * 0.1 for _ in range(3)]
    tabs = (nn.EmbeddingBag(42, h, mode="sum"), nn.EmbeddingBag(13, h, mode="sum"))

    def run(b):
        G = b.collate("edges")
        with torch.no_grad():
            Xv, Xe = tabs[0](G.node_feats), tabs[1](G.edge_feats)
        return _module_forward(G, Xv, Xe, Ws, bs)[2]

    whole = run(batch)
    parts = [run(batch.subset(a, c)) for a, c in ((0, 1000), (1000, 2500), (2500, 4096))]
    assert torch.equal(whole.edge_feats, torch.cat([p.edge_feats for p in parts]))
    assert torch.equal(whole.node_feats, torch.cat([p.node_feats for p in parts]))


def test_determinism_bitexact():
    G = _graph_tensors("qm9", 512, seed=4)
    Xv, Xe = _embed(G, 300)
    torch.manual_seed(0)
    Ws = [torch.randn(300, 300) / 17 for _ in range(3)]
    bs = [torch.randn(300) for _ in range(3)]
    blk, Gd, a = _module_forward(G, Xv, Xe, Ws, bs)
    with torch.no_grad():
        b = blk(Gd)
    assert torch.equal(a.edge_feats, b.edge_feats) and torch.equal(a.node_feats, b.node_feats)


# ------------------------------------------------------------------ contract / errors
def test_forward_contract_and_device_layout_build():
    """A hand-built graph without a collate layout gets its CSR on the device; input not mutated."""
    from notorch_amd.data.models.graph import Graph

    G0 = _graph_tensors("qm9", 8, seed=1)
    Xv, Xe = _embed(G0, 32)
    G = Graph(Xv, Xe, G0.edge_index, G0.rev_index, device_=DEV)
    assert G._nt_layout is None
    torch.manual_seed(0)
    from notorch_amd.nn import ChempropBlock

    blk = ChempropBlock(32, depth=2).to(DEV).eval()
    with torch.no_grad():
        out = blk(G)
    assert out is not G and out.edge_index is G.edge_index and out.rev_index is G.rev_index
    assert G.node_feats.shape == (G0.num_nodes, 32) and torch.equal(G.node_feats.cpu(), Xv)
    Ws, bs = dmpnn_ref.block_params(blk)
    ref_n, ref_e = dmpnn_ref.chemprop_block(Xv, Xe, G0.edge_index, G0.rev_index, Ws, bs)
    assert_parity(out.node_feats, ref_n)


def test_out_of_range_rev_raises_indexerror():
    from notorch_amd.data.models.graph import Graph
    from notorch_amd.nn import ChempropBlock

    Xv, Xe, ei, rev, W, b, _, _ = chain3()
    G = Graph(Xv, Xe, ei, torch.tensor([1, 0, 3, 9]), device_=DEV)
    with pytest.raises(IndexError):
        with torch.no_grad():
            ChempropBlock(2, depth=1).to(DEV)(G)


def test_training_forward_runs_kernels_and_grads_match():
    """Autograd through the block: kernel forward, recompute backward; grads vs oracle autograd."""
    from notorch_amd.nn import ChempropBlock, Sum

    G = _graph_tensors("qm9", 16, seed=6)
    h = 48
    Xv, Xe = _embed(G, h)
    torch.manual_seed(0)
    blk = ChempropBlock(h, depth=2)
    Ws = [l.linear.weight.detach().clone().requires_grad_(True) for l in blk._chemprop_layers()]
    bs = [l.linear.bias.detach().clone().requires_grad_(True) for l in blk._chemprop_layers()]
    Xv_r = Xv.clone().requires_grad_(True)
    n, e = dmpnn_ref.chemprop_block(Xv_r, Xe, G.edge_index, G.rev_index, Ws, bs)
    loss_r = dmpnn_ref.readout(n, G.batch_node_index, len(G)).pow(2).sum() + e.sum()
    loss_r.backward()

    blk = blk.to(DEV).train()
    Xv_d = Xv.to(DEV).requires_grad_(True)
    out = blk(G.update(node_feats=Xv_d, edge_feats=Xe).to(DEV))
    loss = Sum()(out).pow(2).sum() + out.edge_feats.sum()
    loss.backward()
    assert_parity(loss.detach(), loss_r.detach(), what="loss")
    assert_parity(Xv_d.grad, Xv_r.grad, 1e-4, "dXv")
    for l, W in zip(blk._chemprop_layers(), Ws):
        assert_parity(l.linear.weight.grad, W.grad, 1e-4, "dW")


def test_cpu_graph_raises():
    from notorch_amd.nn import ChempropBlock

    Xv, Xe, ei, rev, *_ = chain3()
    from notorch_amd.data.models.graph import Graph

    with pytest.raises(RuntimeError, match="ROCm"):
        ChempropBlock(2, depth=1)(Graph(Xv, Xe, ei, rev))


def test_packed_weight_cache_invalidation():
    """In-place weight updates (optimizer steps) must invalidate the packed MFMA image."""
    from notorch_amd.nn import ChempropBlock

    G = _graph_tensors("qm9", 16, seed=8)
    Xv, Xe = _embed(G, 64)
    torch.manual_seed(0)
    blk = ChempropBlock(64, depth=2).eval()
    Gd = G.update(node_feats=Xv, edge_feats=Xe).to(DEV)
    blk = blk.to(DEV)
    with torch.no_grad():
        blk(Gd)
        for l in blk._chemprop_layers():
            l.linear.weight.mul_(-0.5)
        out = blk(Gd)
    Ws, bs = dmpnn_ref.block_params(blk)
    ref_n, ref_e = dmpnn_ref.chemprop_block(Xv, Xe, G.edge_index, G.rev_index, Ws, bs)
    assert_parity(out.edge_feats, ref_e, what="edge after in-place weight update")


# ------------------------------------------------------------------ load-balanced long segments
@pytest.mark.parametrize("reduce", ["sum", "mean", "max", "min"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_segment_reduce_chunked_skewed(reduce, dtype):
    """nt_segment_reduce_chunked on polymer hubs (in-degree up to ~512) and on 1k-10k-atom molecule
    segments (the readout of config 5), with empty segments mixed in: same result as the oracle up
    to fp32 reassociation at chunk boundaries (max/min exact)."""
    K = _K()
    G = _graph_tensors("polymer", 3, seed=5)
    E, V, h = G.edge_index.shape[1], G.num_nodes, 40
    torch.manual_seed(0)
    X = torch.randn(E, h).to(dtype)
    dst = G.edge_index[1]
    for idx, nseg in ((dst, V + 3), (G.batch_node_index, len(G) + 2)):
        Xs = X if idx is dst else X[:V]
        seg_ptr, perm = K.csr_build(idx.to(DEV), nseg)
        plan = K.chunk_plan(seg_ptr)
        got = K.segment_reduce_chunked(Xs.to(DEV), seg_ptr, perm, nseg, plan, reduce=reduce,
                                       act=K.act_code(nn.ReLU()))
        ref = dmpnn_ref.scatter(torch.relu(Xs.float()), idx, nseg, reduce)
        if dtype == torch.float32:
            tol = 0.0 if reduce in ("max", "min") else 1e-5  # the fp32 contract; sums of up to 10k rows
            assert_parity(got, ref, tol, f"chunked {reduce}")
        else:
            assert_parity(got.float(), ref, 2.0 ** -8, f"chunked bf16 {reduce}")
        assert got[nseg - 1].abs().sum() == 0  # trailing empty segments read 0


@pytest.mark.parametrize("reduce", ["sum", "mean", "max", "min"])
def test_segment_reduce_chunked_without_single_chunk_list(reduce):
    """chunk_seg = NULL (ABI 7): every segment goes through pass 2, as before the single-chunk
    segments were stored by pass 1; the results are the same values."""
    from notorch_amd import _lib
    from notorch_amd.kernels import _ptr, _stream, reduce_code

    K = _K()
    G = _graph_tensors("polymer", 2, seed=6)
    E, V, h = G.edge_index.shape[1], G.num_nodes, 300
    torch.manual_seed(1)
    X = torch.randn(E, h, device=DEV)
    seg_ptr, perm = K.csr_build(G.edge_index[1].to(DEV), V + 2)
    plan = K.chunk_plan(seg_ptr)
    relu = K.act_code(nn.ReLU())
    got = K.segment_reduce_chunked(X, seg_ptr, perm, V + 2, plan, reduce=reduce, act=relu)
    chunk_pos, nchunks, chunk_ptr = plan[:3]
    out = torch.full_like(got, float("nan"))
    partial = torch.empty(nchunks, h, device=DEV)
    rc = _lib.load().nt_segment_reduce_chunked(
        _ptr(X), _ptr(perm), _ptr(chunk_pos), nchunks, _ptr(chunk_ptr), None, None, 0, _ptr(seg_ptr), V + 2, h,
        reduce_code(reduce), relu[0], relu[1], 0, _ptr(partial), _ptr(out), None, _stream(X.device))
    assert rc == 0
    torch.cuda.synchronize()
    assert torch.equal(out, got)


def test_batch_with_zero_bond_molecules():
    """Single-atom molecules (E_i = 0; the reference MolToGraph would crash on them)
    mixed into a batch: their nodes have no in-edge, so S and node rows are 0 (torch_scatter empty
    segment) through the fused zero-filled path, and the readout of such a molecule is 0."""
    from notorch_amd.data.models.graph import BatchedGraph, Graph
    from notorch_amd.data.synth import make_batch
    from notorch_amd.nn import Sum

    Gs = make_batch("qm9", 6, seed=9).to_graphs()
    one = Graph(torch.tensor([[1, 12, 20, 25, 30, 36, 41]]), torch.zeros(0, 2, dtype=torch.long),
                torch.zeros(2, 0, dtype=torch.long), torch.zeros(0, dtype=torch.long))
    G = BatchedGraph.from_graphs([Gs[0], one, Gs[1], Gs[2], one, Gs[3]])
    h = 64
    Xv, Xe = _embed(G, h, seed=4)
    torch.manual_seed(5)
    Ws = [torch.randn(h, h) / 8 for _ in range(3)]
    bs = [torch.randn(h) * 0.1 for _ in range(3)]
    ref_n, ref_e = dmpnn_ref.chemprop_block(Xv, Xe, G.edge_index, G.rev_index, Ws, bs)
    ref_r = dmpnn_ref.readout(ref_n, G.batch_node_index, len(G), "sum")
    _, _, out = _module_forward(G, Xv, Xe, Ws, bs)
    with torch.no_grad():
        r = Sum()(out)
    assert_parity(out.edge_feats, ref_e, what="edge")
    assert_parity(out.node_feats, ref_n, what="node")
    assert_parity(r, ref_r, what="readout")
    assert r[1].abs().sum() == 0 and r[4].abs().sum() == 0


def test_config4_shard_decomposition_bitexact():
    """Config 4 semantics at scale (one GPU's 1M/8 shard is 125k molecules; here 32k split 8 ways):
    the fixed-rev forward of a large batch equals, bit for bit, the concatenation of the forwards of
    its 8 edge-balanced shards (shard.edge_balanced_ranges) — what 8 ranks compute independently."""
    from notorch_amd.data.synth import make_batch
    from notorch_amd.shard import edge_balanced_ranges

    batch = make_batch("qm9", 32768, seed=11)
    h = 300
    torch.manual_seed(1)
    Ws = [torch.randn(h, h) / 17 for _ in range(3)]
    bs = [torch.randn(h) * 0.1 for _ in range(3)]
    tabs = (nn.EmbeddingBag(42, h, mode="sum"), nn.EmbeddingBag(13, h, mode="sum"))

    def run(b):
        G = b.collate("edges")
        with torch.no_grad():
            Xv, Xe = tabs[0](G.node_feats), tabs[1](G.edge_feats)
        return _module_forward(G, Xv, Xe, Ws, bs)[2]

    whole = run(batch)
    ranges = edge_balanced_ranges(2 * batch.n_bonds, 8)
    parts = [run(batch.subset(a, c)) for a, c in ranges]
    assert torch.equal(whole.edge_feats, torch.cat([p.edge_feats for p in parts]))
    assert torch.equal(whole.node_feats, torch.cat([p.node_feats for p in parts]))


@pytest.mark.parametrize("reduce", ["sum", "max"])
def test_all_zero_bond_batch_forward_and_backward(reduce):
    """A batch with no edge at all (E = 0): H is 0 x h, every node row and readout is 0 (empty
    segments, torch_scatter), and the backward gives zero gradients for Xv / weights."""
    from notorch_amd.data.models.graph import BatchedGraph, Graph
    from notorch_amd.nn import ChempropBlock, Sum

    one = Graph(torch.tensor([[1, 12, 20, 25, 30, 36, 41]]), torch.zeros(0, 2, dtype=torch.long),
                torch.zeros(2, 0, dtype=torch.long), torch.zeros(0, dtype=torch.long))
    G = BatchedGraph.from_graphs([one, one, one])
    h = 32
    Xv = torch.randn(G.num_nodes, h, device=DEV, requires_grad=True)
    Xe = torch.zeros(0, h, device=DEV, requires_grad=True)
    blk = ChempropBlock(hidden_dim=h, depth=2, reduce=reduce).to(DEV)
    out = blk(G.to(DEV).update(node_feats=Xv, edge_feats=Xe))
    r = Sum()(out)
    assert out.edge_feats.shape == (0, h) and torch.count_nonzero(out.node_feats) == 0
    assert r.shape == (3, h) and torch.count_nonzero(r) == 0
    r.sum().backward()
    assert torch.count_nonzero(Xv.grad) == 0
    for m in blk._chemprop_layers():
        assert m.linear.weight.grad is None or torch.count_nonzero(m.linear.weight.grad) == 0
