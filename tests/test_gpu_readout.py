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
