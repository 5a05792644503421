"""GPU parity of the attention readouts Gated / SDPAttention (agg.py:50-86):
nt_node_scores + nt_softmax_pool against the oracle's scatter_softmax restatement
(oracle/dmpnn_ref.py readout_gated / readout_sdpa), fp32 normalised max error <= 1e-5; bf16 storage
against the fp32 oracle on the bf16-rounded inputs at 2e-2; gradients through the device-op path."""
import pytest
import torch

from helpers import assert_parity
from oracle import dmpnn_ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _graph(kind="qm9", n=64, seed=0):
    from notorch_amd.data.synth import make_batch

    return make_batch(kind, n, seed=seed).collate("nodes")


@pytest.mark.parametrize("kind,n", [("qm9", 256), ("polymer", 2)])
@pytest.mark.parametrize("h", [300, 13])
def test_gated(kind, n, h):
    from notorch_amd.nn import Gated

    G = _graph(kind, n, seed=1)
    torch.manual_seed(0)
    X = torch.randn(G.num_nodes, h)
    ro = Gated(h)
    ref = dmpnn_ref.readout_gated(X, G.batch_node_index, len(G), ro.a.weight.detach(), ro.a.bias.detach())
    with torch.no_grad():
        got = ro.to(DEV)(G.update(node_feats=X).to(DEV))
    assert got.shape == (len(G), h)
    assert_parity(got, ref, 1e-5, f"Gated {kind}")


@pytest.mark.parametrize("h", [300, 64, 13])
def test_sdpa(h):
    from notorch_amd.nn import SDPAttention

    G = _graph("qm9", 256, seed=2)
    torch.manual_seed(1)
    X = torch.randn(G.num_nodes, h)
    Q = torch.randn(len(G), h)
    ref = dmpnn_ref.readout_sdpa(X, G.batch_node_index, len(G), Q, h ** 0.5)
    with torch.no_grad():
        got = SDPAttention(h)(G.update(node_feats=X).to(DEV), Q=Q.to(DEV))
    assert_parity(got, ref, 1e-5, "SDPAttention")


def test_readouts_bf16():
    from notorch_amd.nn import Gated, SDPAttention

    G = _graph("zinc", 128, seed=3)
    h = 256
    torch.manual_seed(2)
    X = torch.randn(G.num_nodes, h).to(torch.bfloat16)
    Q = torch.randn(len(G), h).to(torch.bfloat16)
    ro = Gated(h).to(torch.bfloat16)
    ref = dmpnn_ref.readout_gated(X.float(), G.batch_node_index, len(G), ro.a.weight.detach().float(),
                                  ro.a.bias.detach().float())
    Gd = G.update(node_feats=X).to(DEV)
    with torch.no_grad():
        got = ro.to(DEV)(Gd)
        got_q = SDPAttention(h)(Gd, Q=Q.to(DEV))
    assert got.dtype == torch.bfloat16
    assert_parity(got.float(), ref, 2e-2, "Gated bf16")
    ref_q = dmpnn_ref.readout_sdpa(X.float(), G.batch_node_index, len(G), Q.float(), h ** 0.5)
    assert_parity(got_q.float(), ref_q, 2e-2, "SDPA bf16")


def test_gated_gradients():
    from notorch_amd.nn import Gated

    G = _graph("qm9", 32, seed=4)
    h = 24
    torch.manual_seed(3)
    X = torch.randn(G.num_nodes, h, dtype=torch.float64)
    ro = Gated(h).double()
    Xr = X.clone().requires_grad_(True)
    dmpnn_ref.readout_gated(Xr, G.batch_node_index, len(G), ro.a.weight, ro.a.bias).pow(2).sum().backward()
    ref_dX, ref_dW = Xr.grad, ro.a.weight.grad.clone()
    ro.zero_grad()
    ro = ro.float().to(DEV)
    Xd = X.float().to(DEV).requires_grad_(True)
    ro(G.update(node_feats=Xd).to(DEV)).pow(2).sum().backward()
    assert_parity(Xd.grad, ref_dX, 1e-5, "dX")
    assert_parity(ro.a.weight.grad, ref_dW, 1e-5, "da")


def test_sdpa_query_gradient_with_frozen_encoder():
    """a learned query with a frozen encoder (X without grad) must still get dL/dQ."""
    from notorch_amd.nn import SDPAttention

    G = _graph("qm9", 32, seed=5)
    h = 24
    torch.manual_seed(4)
    X = torch.randn(G.num_nodes, h, dtype=torch.float64)
    Q = torch.randn(len(G), h, dtype=torch.float64)
    Qr = Q.clone().requires_grad_(True)
    dmpnn_ref.readout_sdpa(X, G.batch_node_index, len(G), Qr, h ** 0.5).pow(2).sum().backward()
    Qd = Q.float().to(DEV).requires_grad_(True)
    out = SDPAttention(h)(G.update(node_feats=X.float()).to(DEV), Q=Qd)
    assert out.grad_fn is not None
    out.pow(2).sum().backward()
    assert_parity(Qd.grad, Qr.grad, 1e-5, "dQ")


@pytest.mark.parametrize("kind,n,h", [("qm9", 256, 300), ("polymer", 2, 64), ("qm9", 16, 13)])
def test_attention_kernel_backward(kind, n, h, monkeypatch):
    """Gated (dX, da, db) and SDPAttention (dX, dQ) through nt_softmax_pool_backward against fp64
    oracle autograd (agg.py:50-86), fp32 contract; the device-op recompute is never called."""
    from notorch_amd.nn import Gated, SDPAttention
    from notorch_amd.nn.gnn import agg

    def _no_torch(*a, **k):
        raise AssertionError("the attention readouts must train on the kernel backward")

    monkeypatch.setattr(agg, "_softmax_pool_torch", _no_torch)
    G = _graph(kind, n, seed=7)
    torch.manual_seed(8)
    X = torch.randn(G.num_nodes, h, dtype=torch.float64)
    w = torch.linspace(-1, 1, h, dtype=torch.float64)
    # Gated
    ro = Gated(h).double()
    Xr = X.clone().requires_grad_(True)
    out = dmpnn_ref.readout_gated(Xr, G.batch_node_index, len(G), ro.a.weight, ro.a.bias)
    (out.pow(2).sum() + (out * w).sum()).backward()
    ref = (Xr.grad, ro.a.weight.grad.clone(), ro.a.bias.grad.clone())
    ro.zero_grad()
    ro = ro.float().to(DEV)
    Xd = X.float().to(DEV).requires_grad_(True)
    o = ro(G.update(node_feats=Xd).to(DEV))
    (o.pow(2).sum() + (o * w.float().to(DEV)).sum()).backward()
    assert_parity(Xd.grad, ref[0], 1e-5, "Gated dX")
    assert_parity(ro.a.weight.grad, ref[1], 1e-5, "Gated da")
    # db = sum_v ds_v is mathematically 0 per molecule (softmax gradients sum to zero): an
    # ill-conditioned difference, held to the fp32 contract relative to the scale of da
    assert (ro.a.bias.grad.double().cpu() - ref[2]).abs().max().item() <= 1e-5 * ref[1].abs().max().item(), "Gated db"
    # SDPAttention: X and Q both trained
    Q = torch.randn(len(G), h, dtype=torch.float64)
    Xr, Qr = X.clone().requires_grad_(True), Q.clone().requires_grad_(True)
    out = dmpnn_ref.readout_sdpa(Xr, G.batch_node_index, len(G), Qr, h ** 0.5)
    (out.pow(2).sum() + (out * w).sum()).backward()
    Xd = X.float().to(DEV).requires_grad_(True)
    Qd = Q.float().to(DEV).requires_grad_(True)
    o = SDPAttention(h)(G.update(node_feats=Xd).to(DEV), Q=Qd)
    (o.pow(2).sum() + (o * w.float().to(DEV)).sum()).backward()
    assert_parity(Xd.grad, Xr.grad, 1e-5, "SDPA dX")
    assert_parity(Qd.grad, Qr.grad, 1e-5, "SDPA dQ")


def test_attention_kernel_backward_bf16():
    """bf16 storage: the kernel gradients stay within 2e-2 (normalised) of fp64 autograd on the
    bf16-rounded inputs."""
    from notorch_amd.nn import Gated

    G = _graph("qm9", 64, seed=9)
    h = 64
    torch.manual_seed(10)
    X = torch.randn(G.num_nodes, h).to(torch.bfloat16)
    ro = Gated(h).to(torch.bfloat16)
    ro64 = Gated(h).double()
    ro64.load_state_dict({k: v.double() for k, v in ro.state_dict().items()})
    Xr = X.double().requires_grad_(True)
    dmpnn_ref.readout_gated(Xr, G.batch_node_index, len(G), ro64.a.weight, ro64.a.bias).pow(2).sum().backward()
    ro = ro.to(DEV)
    Xd = X.to(DEV).requires_grad_(True)
    ro(G.update(node_feats=Xd).to(DEV)).float().pow(2).sum().backward()
    assert Xd.grad.dtype == torch.bfloat16
    assert_parity(Xd.grad.float(), Xr.grad, 2e-2, "Gated bf16 dX")
    assert_parity(ro.a.weight.grad.float(), ro64.a.weight.grad, 2e-2, "Gated bf16 da")
