"""CPU: pin the oracle (restatement) with known-answer tests, fp64 and the committed fixtures."""
import torch

from helpers import FP32_NORM_TOL, assert_parity, chain3, diatomic, load_golden, norm_err
from oracle import dmpnn_ref


def test_kat_chain3():
    # H0 = Xv[src] + Xe = [2,2],[4,-1],[3,-2],[0,0]; M = relu(H0) = [2,2],[4,0],[3,0],[0,0]
    # S[v] = sum of M over in-edges (dst = [1,0,2,1]): S0=[4,0], S1=[2,2], S2=[3,0]
    # A[e] = S[src[e]] - M[rev[e]] (src=[0,1,1,2]): A0=0, A1=0, A2=[2,2], A3=0
    # U = A W^T + b: U2 = [1*2+2*2, 1*2] + b = [6.5, 1]; others = b = [0.5,-1]
    # H1 = H0 + U; node[v] = sum of H1 over in-edges
    Xv, Xe, ei, rev, W, b, H1, node = chain3()
    n, e = dmpnn_ref.chemprop_block(Xv, Xe, ei, rev, [W], [b])
    assert torch.equal(e, H1)
    assert torch.equal(n, node)
    out = dmpnn_ref.readout(n, torch.zeros(3, dtype=torch.long), 1, "sum")
    assert torch.equal(out, torch.tensor([[17.0, -3.0]]))


def test_kat_diatomic_closed_form():
    # every message is S[src] - M[rev] = M[rev] - M[rev] = 0, so H_d = H0 + sum_l b_l exactly
    Xv, Xe, ei, rev, Ws, bs = diatomic()
    n, e = dmpnn_ref.chemprop_block(Xv, Xe, ei, rev, Ws, bs)
    H = Xv[ei[0]] + Xe
    for b in bs:
        H = H + b
    assert torch.equal(e, H)
    assert torch.equal(n, H[[1, 0]])  # node v receives its single in-edge


def test_scatter_semantics():
    x = torch.tensor([[1.0], [5.0], [-2.0], [3.0]])
    idx = torch.tensor([0, 0, 2, 2])
    assert torch.equal(dmpnn_ref.scatter(x, idx, 4, "sum").flatten(), torch.tensor([6.0, 0.0, 1.0, 0.0]))
    assert torch.equal(dmpnn_ref.scatter(x, idx, 4, "mean").flatten(), torch.tensor([3.0, 0.0, 0.5, 0.0]))
    assert torch.equal(dmpnn_ref.scatter(x, idx, 4, "max").flatten(), torch.tensor([5.0, 0.0, 3.0, 0.0]))
    assert torch.equal(dmpnn_ref.scatter(x, idx, 4, "min").flatten(), torch.tensor([1.0, 0.0, -2.0, 0.0]))


def test_golden_fixtures_reproduce():
    for name in ("tiny.npz", "config1.npz"):
        z = load_golden(name)
        t = {k: torch.from_numpy(v) for k, v in z.items()}
        n, e = dmpnn_ref.chemprop_block(
            t["node_feats"], t["edge_feats"], t["edge_index"], t["rev_index"], list(t["W"]), list(t["b"])
        )
        out = dmpnn_ref.readout(n, t["batch_node_index"], int(z["size"]), "sum")
        assert_parity(n, t["out_node"], 1e-6, name)
        assert_parity(e, t["out_edge"], 1e-6, name)
        assert_parity(out, t["out_sum"], 1e-6, name)
        # the fp32 restatement sits within the fp32 contract of the fp64 truth
        assert norm_err(out, t["out_sum64"]) <= FP32_NORM_TOL


def test_fp32_vs_fp64_noise_floor():
    z = load_golden("config1.npz")
    assert z["err64_node"] / abs(z["out_node"]).max() <= FP32_NORM_TOL
    assert z["err64_edge"] / abs(z["out_edge"]).max() <= FP32_NORM_TOL


def test_scatter_softmax_hand_case():
    """torch_scatter scatter_softmax restatement on a hand-checkable case (molecules {0,1,2}, {3},
    {} ): each molecule's weights are a softmax of its own scores, an empty molecule gets none."""
    import math

    s = torch.tensor([0.0, math.log(2.0), math.log(3.0), 5.0])
    idx = torch.tensor([0, 0, 0, 1])
    got = dmpnn_ref.scatter_softmax(s, idx, 3)
    assert torch.allclose(got, torch.tensor([1 / 6, 2 / 6, 3 / 6, 1.0]), atol=1e-7)
    X = torch.tensor([[6.0, 0.0], [0.0, 6.0], [6.0, 6.0], [1.0, 2.0]])
    out = dmpnn_ref.readout_gated(X, idx, 3, torch.zeros(1, 2), torch.zeros(1))  # uniform alpha
    assert torch.allclose(out, torch.tensor([[4.0, 4.0], [1.0, 2.0], [0.0, 0.0]]))
    Q = torch.tensor([[0.0, 0.0], [1.0, 1.0], [0.0, 0.0]])
    out = dmpnn_ref.readout_sdpa(X, idx, 3, Q, 2.0)  # molecule 0: Q = 0 -> uniform
    assert torch.allclose(out, torch.tensor([[4.0, 4.0], [1.0, 2.0], [0.0, 0.0]]))
