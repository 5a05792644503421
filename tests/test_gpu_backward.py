"""GPU parity of the training path: kernel backward (csrc/backward.hip + library GEMMs) against
the CPU oracle's autograd (oracle/dmpnn_ref.py, i.e. ATen autograd of chemprop.py:28-88 and
agg.py:23-38).

Criterion: gradients are compared with the fp64 oracle autograd as the truth, normalised max error
<= GRAD_TOL.  The fp32 oracle itself sits at ~1e-7..1e-6 of fp64 on these cases; GRAD_TOL leaves
room for the different (but fp32) accumulation orders of the GEMM library and the segment sums.
"""
import pytest
import torch
import torch.nn as nn

from helpers import assert_parity, norm_err
from oracle import dmpnn_ref

pytestmark = pytest.mark.gpu

DEV = "cuda"
GRAD_TOL = 1e-5


def _graph(kind="qm9", n=16, seed=0, rev_offset="nodes"):
    from notorch_amd.data.synth import make_batch

    return make_batch(kind, n, seed=seed).collate(rev_offset)


def _embed(G, h, seed=0):
    torch.manual_seed(seed)
    nt = nn.EmbeddingBag(42, h, mode="sum")
    et = nn.EmbeddingBag(13, h, mode="sum")
    with torch.no_grad():
        return nt(G.node_feats), et(G.edge_feats)


_ACTS = {"ReLU": (nn.ReLU, torch.relu), "Identity": (nn.Identity, lambda x: x),
         "SiLU": (nn.SiLU, torch.nn.functional.silu), "Tanh": (nn.Tanh, torch.tanh),
         "ELU": (nn.ELU, torch.nn.functional.elu), "GELU": (nn.GELU, torch.nn.functional.gelu)}


def _oracle_grads(G, Xv, Xe, blk, act_fn, residual, reduce, readout, dtype):
    Ws, bs = dmpnn_ref.block_params(blk)
    Ws = [W.detach().to(dtype, copy=True).requires_grad_(True) for W in Ws]
    bs = [None if b is None else b.detach().to(dtype, copy=True).requires_grad_(True) for b in bs]
    Xv_r = Xv.detach().to(dtype, copy=True).requires_grad_(True)
    Xe_r = Xe.detach().to(dtype, copy=True).requires_grad_(True)
    n, e = dmpnn_ref.chemprop_block(Xv_r, Xe_r, G.edge_index, G.rev_index, Ws, bs, act=act_fn,
                                    residual=residual, reduce=reduce)
    r = dmpnn_ref.readout(n, G.batch_node_index, len(G), readout)
    loss = r.pow(2).sum() + (e * torch.linspace(-1, 1, e.shape[1], dtype=dtype)).sum()
    loss.backward()
    return loss.detach(), Xv_r.grad, Xe_r.grad, [W.grad for W in Ws], [None if b is None else b.grad for b in bs]


def _device_grads(G, Xv, Xe, blk, readout):
    from notorch_amd.nn import Max, Mean, Min, Sum

    blk = blk.to(DEV).train()
    Xv_d = Xv.to(DEV).requires_grad_(True)
    Xe_d = Xe.to(DEV).requires_grad_(True)
    out = blk(G.update(node_feats=Xv_d, edge_feats=Xe_d).to(DEV))
    ro = {"sum": Sum, "mean": Mean, "max": Max, "min": Min}[readout]()(out)
    e = out.edge_feats
    loss = ro.pow(2).sum() + (e * torch.linspace(-1, 1, e.shape[1], device=DEV)).sum()
    loss.backward()
    layers = blk._chemprop_layers()
    return (loss.detach(), Xv_d.grad, Xe_d.grad, [l.linear.weight.grad for l in layers],
            [None if l.linear.bias is None else l.linear.bias.grad for l in layers])


def _check(G, h, depth=2, act="ReLU", residual=True, reduce="sum", readout="sum", bias=True,
           shared=False, tol=GRAD_TOL, fp32_floor=False):
    """fp32_floor: the tolerance becomes max(tol, 4 x the fp32 oracle's own error vs fp64) — for
    graphs whose long segment sums (polymer hubs) put the fp32 noise floor itself above tol."""
    from notorch_amd.nn import ChempropBlock

    Xv, Xe = _embed(G, h)
    torch.manual_seed(1)
    blk = ChempropBlock(h, act=_ACTS[act][0], bias=bias, depth=depth, residual=residual,
                        shared=shared, reduce=reduce)
    truth = _oracle_grads(G, Xv, Xe, blk, _ACTS[act][1], residual, reduce, readout, torch.float64)
    if fp32_floor:
        o32 = _oracle_grads(G, Xv, Xe, blk, _ACTS[act][1], residual, reduce, readout, torch.float32)
        floor = max(norm_err(a, b) for a, b in zip(o32[1:3] + tuple(o32[3]), truth[1:3] + tuple(truth[3])))
        tol = max(tol, 4 * floor)
    got = _device_grads(G, Xv, Xe, blk, readout)
    assert_parity(got[0], truth[0], tol, "loss")
    assert_parity(got[1], truth[1], tol, "dXv")
    assert_parity(got[2], truth[2], tol, "dXe")
    if shared:  # one parameter repeated: its grad is the sum over layers
        truth_W = [sum(truth[3])]
        truth_b = [sum(truth[4])] if bias else [None]
        got_W, got_b = got[3][:1], got[4][:1]
    else:
        truth_W, truth_b, got_W, got_b = truth[3], truth[4], got[3], got[4]
    for l, (a, b) in enumerate(zip(got_W, truth_W)):
        assert_parity(a, b, tol, f"dW[{l}]")
    for l, (a, b) in enumerate(zip(got_b, truth_b)):
        if b is None:
            assert a is None
        else:
            assert_parity(a, b, tol, f"db[{l}]")


# ------------------------------------------------------------------ kernels one by one
def test_message_kernel():
    from notorch_amd import kernels as K

    G = _graph("qm9", 8, seed=1)
    E, V, h = G.num_edges, G.num_nodes, 36
    torch.manual_seed(0)
    H, S = torch.randn(E, h), torch.randn(V, h)
    src, rev = G.edge_index[0], G.rev_index
    ref = S[src] - torch.relu(H[rev])
    got = K.dmpnn_message(H.to(DEV), S.to(DEV), src.to(DEV), rev.to(DEV))
    assert torch.equal(got.cpu(), ref)  # one subtraction per element: bit-exact


@pytest.mark.parametrize("h", [16, 30])  # float4 and scalar paths
@pytest.mark.parametrize("reduce", ["sum", "mean"])
def test_edge_backward_kernel(h, reduce):
    from notorch_amd import kernels as K

    G = _graph("qm9", 8, seed=2)  # reference collate: rev_index is not a permutation
    E, V = G.num_edges, G.num_nodes
    torch.manual_seed(0)
    Gr, H, dA, dS = torch.randn(E, h), torch.randn(E, h), torch.randn(E, h), torch.randn(V, h)
    src, dst, rev = G.edge_index[0], G.edge_index[1], G.rev_index
    cnt = torch.zeros(V).index_add_(0, dst, torch.ones(E)).clamp(min=1)
    scale = (1.0 / cnt) if reduce == "mean" else torch.ones(V)
    dM = (dS * scale[:, None])[dst] - torch.zeros(E, h, dtype=torch.float64).index_add_(
        0, rev, dA.double()).float()
    ref = Gr + (H > 0).float() * dM
    Gd = G.to(DEV)
    dst_ptr, _ = K.csr_build(dst.to(DEV), V)
    rev_ptr, rev_perm = K.csr_build(rev.to(DEV), E)
    got = K.dmpnn_edge_backward(Gr.to(DEV), H.to(DEV), dA.to(DEV), dS.to(DEV), Gd.edge_index[1].contiguous(),
                                rev_ptr, rev_perm, dst_ptr, reduce=reduce)
    assert_parity(got, ref, 1e-6, "edge backward")


def test_gather_rows_kernel():
    from notorch_amd import kernels as K

    torch.manual_seed(0)
    X = torch.randn(5, 12)
    idx = torch.tensor([0, 0, 3, 4, 4, 4, 1])
    base = torch.randn(7, 12)
    seg_ptr = torch.tensor([0, 2, 3, 3, 4, 7], dtype=torch.int32)  # counts 2,1,0,1,3
    cnt = (seg_ptr[1:] - seg_ptr[:-1]).clamp(min=1).float()
    got = K.gather_rows(X.to(DEV), idx.to(DEV), base=base.to(DEV), seg_ptr=seg_ptr.to(DEV))
    assert_parity(got, base + X[idx] / cnt[idx][:, None], 1e-7, "gather mean")
    got = K.gather_rows(X.to(DEV), idx.to(DEV))
    assert torch.equal(got.cpu(), X[idx])


# ------------------------------------------------------------------ block + readout gradients
@pytest.mark.parametrize("reduce,readout", [("sum", "sum"), ("mean", "mean"), ("sum", "mean")])
def test_block_grads_reduce(reduce, readout):
    _check(_graph("qm9", 16, seed=6), 48, depth=3, reduce=reduce, readout=readout)


@pytest.mark.parametrize("act", ["ReLU", "Identity", "SiLU", "Tanh", "ELU", "GELU"])
def test_block_grads_act(act):
    _check(_graph("qm9", 12, seed=7), 32, depth=2, act=act)


@pytest.mark.parametrize("opts", [dict(residual=False), dict(bias=False), dict(shared=True, depth=3),
                                  dict(depth=1), dict(depth=5)])
def test_block_grads_options(opts):
    _check(_graph("qm9", 12, seed=8), 40, **opts)


def test_block_grads_fixed_rev():
    _check(_graph("qm9", 12, seed=9, rev_offset="edges"), 40, depth=3)


def test_block_grads_odd_hidden_scalar_path():
    _check(_graph("qm9", 8, seed=10), 13, depth=2)


def test_block_grads_polymer_hubs_unfused_forward():
    # in-degree up to ~512: the forward takes the unfused update + segment_reduce path.  Sums over
    # 512-edge hubs make the sum-reduce gradients ill-conditioned (the fp32 oracle alone is ~1e-3
    # off fp64), so the hub graph runs with mean aggregation and readout, and the fp32 floor guard.
    _check(_graph("polymer", 2, seed=11), 32, depth=2, reduce="mean", readout="mean", fp32_floor=True)


def _rel_l2(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


@pytest.mark.parametrize("act", ["ReLU", "SiLU"])
def test_block_grads_config2_fp32(act):
    """Config-2 shape (4096 QM9 molecules, h=300, depth 3), fp64 oracle autograd as the truth.

    SiLU (smooth): every gradient within the fp32 contract of fp64, normalised max <= 1e-5.
    ReLU: at 23M edge-state elements some H_l entries sit within fp32 rounding of 0, so ANY two
    fp32 evaluations disagree on relu'(H) there and the gradient of that element (and, through the
    earlier layers, of its molecule) jumps by a whole dm.  Measured on MI355X: the fp32 CPU oracle
    itself is 1.2e-2 (max) / 1.4e-4 (L2) off fp64 on dXv, the kernels 1.2e-2 / 1.3e-4 (and
    3e-7 / 3e-7 with SiLU).  So for ReLU the kernels must be no further from fp64 than 2x the fp32
    CPU oracle, on both the normalised max and the relative L2 error (tools/diag_grad.py)."""
    from notorch_amd.nn import ChempropBlock

    G = _graph("qm9", 4096, seed=0)
    h = 300
    Xv, Xe = _embed(G, h)
    torch.manual_seed(1)
    blk = ChempropBlock(h, depth=3, act=_ACTS[act][0])
    fn = _ACTS[act][1]
    truth = _oracle_grads(G, Xv, Xe, blk, fn, True, "sum", "sum", torch.float64)
    o32 = _oracle_grads(G, Xv, Xe, blk, fn, True, "sum", "sum", torch.float32)
    got = _device_grads(G, Xv, Xe, blk, "sum")
    pairs = [("dXv", got[1], o32[1], truth[1]), ("dXe", got[2], o32[2], truth[2])]
    pairs += [(f"dW[{l}]", a, c, b) for l, (a, c, b) in enumerate(zip(got[3], o32[3], truth[3]))]
    pairs += [(f"db[{l}]", a, c, b) for l, (a, c, b) in enumerate(zip(got[4], o32[4], truth[4]))]
    for name, a, c, b in pairs:
        if act == "SiLU":
            assert_parity(a, b, GRAD_TOL, name)
            continue
        l2, l2_cpu = _rel_l2(a, b), _rel_l2(c, b)
        assert l2 <= max(1e-5, 2 * l2_cpu), f"{name}: relative L2 {l2:.3e} (fp32 CPU oracle {l2_cpu:.3e})"
        assert_parity(a, b, max(2e-5, 2 * norm_err(c, b)), name)


@pytest.mark.parametrize("reduce,readout,act", [("max", "sum", "SiLU"), ("min", "max", "Tanh"),
                                                ("max", "min", "Identity"), ("max", "max", "ReLU")])
def test_max_min_kernel_backward(reduce, readout, act, monkeypatch):
    """fp32 max / min aggregations and Max / Min readouts train through the arg kernels
    (nt_segment_arg + nt_dmpnn_edge_backward_arg + nt_gather_rows_arg; torch_scatter's scatter_max
    / scatter_min gradient at chemprop.py:39,86 and agg.py:45), never through the torch recompute."""
    from notorch_amd.nn.gnn import _engine

    def boom(*a, **k):
        raise AssertionError("fp32 max/min backward must use the kernel path")

    monkeypatch.setattr(_engine, "_torch_block", boom)
    monkeypatch.setattr(_engine, "_torch_scatter", boom)
    _check(_graph("qm9", 12, seed=12), 24, depth=2, reduce=reduce, readout=readout, act=act)


def test_max_reduce_recompute_backward_still_exact(monkeypatch):
    """NT_BWD=torch (the recompute path, which bf16 max / min still take) agrees with the oracle."""
    monkeypatch.setenv("NT_BWD", "torch")
    _check(_graph("qm9", 8, seed=12), 24, depth=2, reduce="max")


def test_segment_arg_first_occurrence():
    """Ties go to the first row in ascending CSR order (torch_scatter's CPU reducer: strict > / <);
    empty segments get -1."""
    from notorch_amd import kernels as K

    X = torch.tensor([[1.0, 5.0], [3.0, 5.0], [3.0, -1.0], [0.0, 2.0]], device=DEV)
    seg_ptr = torch.tensor([0, 3, 3, 4], dtype=torch.int32, device=DEV)  # segments {0,1,2}, {}, {3}
    perm = torch.tensor([2, 0, 1, 3], dtype=torch.int32, device=DEV)     # visiting order 2, 0, 1
    a_max = K.segment_arg(X, seg_ptr, perm, 3, "max").cpu().tolist()
    a_min = K.segment_arg(X, seg_ptr, perm, 3, "min").cpu().tolist()
    assert a_max == [[2, 0], [-1, -1], [3, 3]]
    assert a_min == [[0, 2], [-1, -1], [3, 3]]


def test_backward_does_not_route_through_torch_block_for_sum(monkeypatch):
    from notorch_amd.nn.gnn import _engine

    def boom(*a, **k):
        raise AssertionError("sum-reduce backward must use the kernel path")

    monkeypatch.setattr(_engine, "_torch_block", boom)
    _check(_graph("qm9", 8, seed=13), 32, depth=2)


@pytest.mark.parametrize("uses", ["node", "edge"])
def test_block_grads_one_output_unused(uses):
    """A loss on one of the block's two outputs only: the other's gradient arrives as None (the
    Function does not materialise zeros), and the backward starts from the used one alone."""
    from notorch_amd.nn import ChempropBlock, Sum

    G = _graph("qm9", 24, seed=7)
    h = 64
    Xv, Xe = _embed(G, h)
    torch.manual_seed(2)
    blk = ChempropBlock(h, depth=3)
    Ws, bs = dmpnn_ref.block_params(blk)
    Ws = [W.detach().double().requires_grad_(True) for W in Ws]
    bs = [b.detach().double().requires_grad_(True) for b in bs]
    Xv_r, Xe_r = Xv.double().requires_grad_(True), Xe.double().requires_grad_(True)
    n, e = dmpnn_ref.chemprop_block(Xv_r, Xe_r, G.edge_index, G.rev_index, Ws, bs)
    w = torch.linspace(-1, 1, h, dtype=torch.float64)
    loss = dmpnn_ref.readout(n, G.batch_node_index, len(G), "sum").pow(2).sum() if uses == "node" \
        else (e * w).sum()
    loss.backward()
    blk = blk.to(DEV).train()
    Xv_d, Xe_d = Xv.to(DEV).requires_grad_(True), Xe.to(DEV).requires_grad_(True)
    out = blk(G.update(node_feats=Xv_d, edge_feats=Xe_d).to(DEV))
    dloss = Sum()(out).pow(2).sum() if uses == "node" else (out.edge_feats * w.float().to(DEV)).sum()
    dloss.backward()
    assert_parity(Xv_d.grad, Xv_r.grad, GRAD_TOL, "dXv")
    assert_parity(Xe_d.grad, Xe_r.grad, GRAD_TOL, "dXe")
    for l, (m, W) in enumerate(zip(blk._chemprop_layers(), Ws)):
        assert_parity(m.linear.weight.grad, W.grad, GRAD_TOL, f"dW[{l}]")
