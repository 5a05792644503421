"""bf16 kernel backward (csrc/backward.hip bf16 kernels; engine block_backward with bf16 storage).

bf16 has no bit-exact target: every stored edge/node state is rounded to 8 mantissa bits, so a
bf16 gradient differs from the fp64 truth by the rounding the forward and backward states carry.
The contract, per gradient tensor:
* the kernel gradients are no further from the fp64 oracle (reference chemprop.py / residual.py,
  restated in oracle/dmpnn_ref.py, on the same bf16-valued inputs and weights) than
  ``BF16_FACTOR`` x the reference's own bf16 autograd run on the same device (the torch-op
  recompute, NT_BWD=torch), or than the absolute floor ``BF16_FLOOR``, on both the normalised max
  error and the relative L2 error;
* the element kernels are checked against an fp32 restatement of the same formula with a
  one-ulp (2^-8 normalised) tolerance.
"""
import pytest
import torch
import torch.nn as nn

from helpers import assert_parity, norm_err
from oracle import dmpnn_ref

pytestmark = pytest.mark.gpu

DEV = "cuda"
BF16 = torch.bfloat16
ULP = 2.0 ** -8
BF16_FACTOR = 2.0
BF16_FLOOR = 2e-2


def _graph(kind="qm9", n=16, seed=0):
    from notorch_amd.data.synth import make_batch

    return make_batch(kind, n, seed=seed).collate("nodes")


def _rel_l2(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


# ------------------------------------------------------------------ element kernels
@pytest.mark.parametrize("h", [64, 36])  # 16-B piece and scalar paths
def test_message_bf16(h):
    from notorch_amd import kernels as K

    G = _graph("qm9", 8, seed=1)
    E, V = G.num_edges, G.num_nodes
    torch.manual_seed(0)
    H, S = torch.randn(E, h).to(BF16), torch.randn(V, h).to(BF16)
    src, rev = G.edge_index[0], G.rev_index
    ref = (S.float()[src] - torch.relu(H.float()[rev])).to(BF16)  # one fp32 op, one rounding
    got = K.dmpnn_message(H.to(DEV), S.to(DEV), src.to(DEV), rev.to(DEV))
    assert got.dtype == BF16
    assert torch.equal(got.cpu(), ref)


@pytest.mark.parametrize("h", [64, 36])
@pytest.mark.parametrize("reduce", ["sum", "mean"])
def test_edge_backward_bf16(h, reduce):
    from notorch_amd import kernels as K

    G = _graph("qm9", 8, seed=2)
    E, V = G.num_edges, G.num_nodes
    torch.manual_seed(0)
    Gr, H, dA, dS = (torch.randn(E, h).to(BF16), torch.randn(E, h).to(BF16),
                     torch.randn(E, h).to(BF16), torch.randn(V, h).to(BF16))
    src, dst, rev = G.edge_index[0], G.edge_index[1], G.rev_index
    cnt = torch.zeros(V).index_add_(0, dst, torch.ones(E)).clamp(min=1)
    scale = (1.0 / cnt) if reduce == "mean" else torch.ones(V)
    dM = (dS.float() * scale[:, None])[dst] - torch.zeros(E, h).index_add_(0, rev, dA.float())
    ref = Gr.float() + (H.float() > 0).float() * dM
    dst_ptr, _ = K.csr_build(dst.to(DEV), V)
    rev_ptr, rev_perm = K.csr_build(rev.to(DEV), E)
    got = K.dmpnn_edge_backward(Gr.to(DEV), H.to(DEV), dA.to(DEV), dS.to(DEV), dst.to(DEV),
                                rev_ptr, rev_perm, dst_ptr, reduce=reduce)
    assert got.dtype == BF16
    assert_parity(got.float(), ref, ULP, "edge backward bf16")


def test_gather_rows_bf16():
    from notorch_amd import kernels as K

    torch.manual_seed(0)
    X = torch.randn(5, 16).to(BF16)
    idx = torch.tensor([0, 0, 3, 4, 4, 4, 1])
    base = torch.randn(7, 16).to(BF16)
    seg_ptr = torch.tensor([0, 2, 3, 3, 4, 7], dtype=torch.int32)
    cnt = (seg_ptr[1:] - seg_ptr[:-1]).clamp(min=1).float()
    got = K.gather_rows(X.to(DEV), idx.to(DEV), base=base.to(DEV), seg_ptr=seg_ptr.to(DEV))
    assert_parity(got.float(), base.float() + X.float()[idx] / cnt[idx][:, None], ULP, "gather mean bf16")
    got = K.gather_rows(X.to(DEV), idx.to(DEV))
    assert torch.equal(got.cpu(), X[idx])


# ------------------------------------------------------------------ block gradients
def _truth(G, Xv, Xe, blk, act_fn, reduce):
    Ws, bs = dmpnn_ref.block_params(blk)
    Ws = [W.detach().double().requires_grad_(True) for W in Ws]
    bs = [None if b is None else b.detach().double().requires_grad_(True) for b in bs]
    Xv_r = Xv.detach().double().requires_grad_(True)
    Xe_r = Xe.detach().double().requires_grad_(True)
    n, e = dmpnn_ref.chemprop_block(Xv_r, Xe_r, G.edge_index, G.rev_index, Ws, bs, act=act_fn,
                                    residual=True, reduce=reduce)
    r = dmpnn_ref.readout(n, G.batch_node_index, len(G), reduce)
    loss = r.pow(2).sum() + (e * torch.linspace(-1, 1, e.shape[1], dtype=torch.float64)).sum()
    loss.backward()
    return [Xv_r.grad, Xe_r.grad] + [W.grad for W in Ws] + [b.grad for b in bs]


def _device(G, Xv, Xe, blk, reduce, mode, monkeypatch):
    from notorch_amd.nn import Max, Mean, Min, Sum

    monkeypatch.setenv("NT_BWD", mode)
    for p in blk.parameters():
        p.grad = None
    Xv_d = Xv.to(DEV).requires_grad_(True)
    Xe_d = Xe.to(DEV).requires_grad_(True)
    out = blk(G.update(node_feats=Xv_d, edge_feats=Xe_d).to(DEV))
    ro = {"sum": Sum, "mean": Mean, "max": Max, "min": Min}[reduce]()(out)
    e = out.edge_feats.float()
    loss = ro.float().pow(2).sum() + (e * torch.linspace(-1, 1, e.shape[1], device=DEV)).sum()
    loss.backward()
    layers = blk._chemprop_layers()
    return ([Xv_d.grad, Xe_d.grad] + [l.linear.weight.grad for l in layers]
            + [l.linear.bias.grad for l in layers])


@pytest.mark.parametrize("kind,n,h,depth,act,reduce", [
    ("qm9", 64, 64, 3, "ReLU", "sum"),
    ("qm9", 64, 64, 3, "SiLU", "mean"),
    ("qm9", 32, 36, 2, "ReLU", "sum"),       # h % 8 != 0: unfused update, scalar element kernels
    ("zinc", 256, 512, 5, "ReLU", "sum"),    # config-3 shape at a smaller batch (fused bf16 update)
    ("qm9", 64, 64, 3, "ReLU", "max"),       # max / min: the arg kernels on bf16 storage
    ("qm9", 32, 36, 2, "SiLU", "min"),
])
def test_block_grads_bf16(kind, n, h, depth, act, reduce, monkeypatch):
    from notorch_amd.nn import ChempropBlock
    from notorch_amd.nn.gnn import _engine

    acts = {"ReLU": (nn.ReLU, torch.relu), "SiLU": (nn.SiLU, torch.nn.functional.silu)}
    G = _graph(kind, n, seed=3)
    torch.manual_seed(0)
    Xv = nn.EmbeddingBag(42, h, mode="sum")(G.node_feats).detach().to(BF16)
    Xe = nn.EmbeddingBag(13, h, mode="sum")(G.edge_feats).detach().to(BF16)
    torch.manual_seed(1)
    blk = ChempropBlock(h, depth=depth, act=acts[act][0], reduce=reduce).to(DEV, BF16).train()
    truth = _truth(G, Xv, Xe, blk, acts[act][1], reduce)

    calls = []
    real = _engine.block_backward
    monkeypatch.setattr(_engine, "block_backward", lambda *a, **k: calls.append(1) or real(*a, **k))
    got = _device(G, Xv, Xe, blk, reduce, "kernel", monkeypatch)
    assert calls, "bf16 backward must take the kernel path (every reduce)"
    ref = _device(G, Xv, Xe, blk, reduce, "torch", monkeypatch)
    names = ["dXv", "dXe"] + [f"dW[{l}]" for l in range(depth)] + [f"db[{l}]" for l in range(depth)]
    for name, a, r, t in zip(names, got, ref, truth):
        assert a.dtype == BF16, name
        assert torch.isfinite(a.float()).all(), name
        e_max, r_max = norm_err(a.float(), t), norm_err(r.float(), t)
        e_l2, r_l2 = _rel_l2(a, t), _rel_l2(r, t)
        print(f"{name}: kernel max {e_max:.2e} l2 {e_l2:.2e} | torch bf16 max {r_max:.2e} l2 {r_l2:.2e}")
        assert e_max <= max(BF16_FLOOR, BF16_FACTOR * r_max), f"{name}: max {e_max:.3e} vs torch bf16 {r_max:.3e}"
        assert e_l2 <= max(BF16_FLOOR, BF16_FACTOR * r_l2), f"{name}: L2 {e_l2:.3e} vs torch bf16 {r_l2:.3e}"


@pytest.mark.parametrize("h,E,act", [(512, 20_000, "relu"), (64, 4097, "identity"), (128, 33, "gelu"),
                                     (96, 1, "relu"), (400, 3000, "tanh")])
def test_weight_grad_bf16(h, E, act):
    """nt_dmpnn_weight_grad on bf16 storage (config 3's dW = G^T A, db = colsum G): A formed in fp32
    and rounded to bf16 once (bit-identical to nt_dmpnn_message), exact bf16 products, fp32
    accumulation: within the fp32 contract of the fp64 product of the same bf16 operands; repeat
    bit-identical."""
    from helpers import FP32_NORM_TOL
    from notorch_amd import kernels as K

    mods = {"relu": nn.ReLU(), "identity": nn.Identity(), "gelu": nn.GELU(), "tanh": nn.Tanh()}
    mod = mods[act]
    g = torch.Generator().manual_seed(E + h)
    V = max(E // 2, 1)
    Gr = torch.randn(E, h, generator=g).to(BF16)
    H, S = torch.randn(E, h, generator=g).to(BF16), torch.randn(V, h, generator=g).to(BF16)
    src = torch.randint(0, V, (E,), generator=g)
    rev = torch.randint(0, E, (E,), generator=g)
    args = (Gr.to(DEV), H.to(DEV), S.to(DEV), src.to(DEV), rev.to(DEV))
    dW, db = K.weight_grad(*args, act=K.act_code(mod))
    A = K.dmpnn_message(args[1], args[2], args[3], args[4], act=K.act_code(mod)).cpu()  # bf16 message
    assert dW.dtype == torch.float32
    assert_parity(dW, Gr.double().t() @ A.double(), FP32_NORM_TOL, f"dW h={h} E={E} {act}")
    assert_parity(db, Gr.double().sum(0), FP32_NORM_TOL, f"db h={h} E={E}")
    dW2, db2 = K.weight_grad(*args, act=K.act_code(mod))
    assert torch.equal(dW, dW2) and torch.equal(db, db2)


@pytest.mark.parametrize("h,M", [(512, 20_000), (64, 100), (200, 7)])
def test_dense_matmul_bf16(h, M):
    """dA = G W on the bf16 layer kernel's dense mode: fp32 accumulation of exact bf16 products,
    one rounding (within one bf16 ulp of the fp64 product, normalised)."""
    from notorch_amd import kernels as K

    g = torch.Generator().manual_seed(M + h)
    X = torch.randn(M, h, generator=g).to(BF16)
    W = (torch.randn(h, h, generator=g) / h ** 0.5).to(BF16)
    out = K.dense_matmul(X.to(DEV), K.pack_weights(W.t().contiguous().to(DEV)))
    assert out.dtype == BF16
    assert_parity(out, X.double() @ W.double(), ULP, f"dense bf16 h={h} M={M}")
