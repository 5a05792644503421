"""Shared test helpers: tolerance criterion and hand-checkable graphs."""
import numpy as np
import torch

# Parity criterion: normalised max error max|a - b| / max|b| <= 1e-5 for fp32.
FP32_NORM_TOL = 1e-5


def norm_err(a: torch.Tensor, b: torch.Tensor) -> float:
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    if b.numel() == 0:
        return 0.0
    scale = b.abs().max().item()
    return (a - b).abs().max().item() / (scale if scale > 0 else 1.0)


def assert_parity(a, b, tol=FP32_NORM_TOL, what=""):
    assert a.shape == b.shape, f"{what}: shape {tuple(a.shape)} != {tuple(b.shape)}"
    e = norm_err(a, b)
    assert e <= tol, f"{what}: normalised max error {e:.3e} > {tol:.1e}"


def chain3():
    """3-atom chain 0-1-2 in MolToGraph layout (bond b -> edges 2b, 2b+1; rev = [1,0,3,2])."""
    Xv = torch.tensor([[1.0, 2.0], [3.0, -1.0], [0.0, 1.0]])
    Xe = torch.tensor([[1.0, 0.0], [1.0, 0.0], [0.0, -1.0], [0.0, -1.0]])
    edge_index = torch.tensor([[0, 1, 1, 2], [1, 0, 2, 1]])
    rev = torch.tensor([1, 0, 3, 2])
    W = torch.tensor([[1.0, 2.0], [0.0, 1.0]])
    b = torch.tensor([0.5, -1.0])
    # hand-derived (see tests/test_oracle.py::test_kat_chain3 for the derivation)
    H1 = torch.tensor([[2.5, 1.0], [4.5, -2.0], [9.5, -1.0], [0.5, -1.0]])
    node = torch.tensor([[4.5, -2.0], [3.0, 0.0], [9.5, -1.0]])
    return Xv, Xe, edge_index, rev, W, b, H1, node


def diatomic(h=8, depth=3, seed=0):
    g = torch.Generator().manual_seed(seed)
    Xv = torch.randn(2, h, generator=g)
    Xe = torch.randn(1, h, generator=g).repeat(2, 1)
    edge_index = torch.tensor([[0, 1], [1, 0]])
    rev = torch.tensor([1, 0])
    Ws = [torch.randn(h, h, generator=g) for _ in range(depth)]
    bs = [torch.randn(h, generator=g) for _ in range(depth)]
    return Xv, Xe, edge_index, rev, Ws, bs


def load_golden(name):
    import os

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", name)
    return dict(np.load(path, allow_pickle=False))
