"""hipGraph capture of the forward (notorch_amd/graphs.py): a replay is bit-identical to the eager
forward, recomputes on refilled inputs, and covers the fp32 fused, bf16 and embedded encoders."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _case(n=32, h=300, dtype=torch.float32, seed=0):
    from notorch_amd.data.synth import make_batch
    from notorch_amd.nn import ChempropBlock, Sum

    G = make_batch("qm9", n, seed=seed).collate("nodes")
    torch.manual_seed(seed)
    Xv = torch.randn(G.num_nodes, h).to(dtype)
    Xe = torch.randn(G.num_edges, h).to(dtype)
    blk = ChempropBlock(hidden_dim=h, depth=3).eval().to(dtype).to(DEV)
    return G.update(node_feats=Xv, edge_feats=Xe).to(DEV), blk, Sum()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_graphed_forward_matches_eager_and_recomputes(dtype):
    from notorch_amd.graphs import GraphedForward

    Gd, blk, ro = _case(dtype=dtype)
    fn = lambda G: ro(blk(G))  # noqa: E731
    with torch.no_grad():
        eager = fn(Gd).clone()
    fwd = GraphedForward(fn, Gd)
    assert torch.equal(fwd(), eager)
    G2 = Gd.update(node_feats=torch.randn_like(Gd.node_feats.float()).to(dtype),
                   edge_feats=torch.randn_like(Gd.edge_feats.float()).to(dtype))
    with torch.no_grad():
        eager2 = fn(G2).clone()
    fwd.copy_inputs(G2)
    assert torch.equal(fwd(), eager2)
    assert not torch.equal(eager, eager2)


def test_graphed_embedded_encoder():
    from notorch_amd.data.synth import make_batch
    from notorch_amd.graphs import GraphedForward
    from notorch_amd.nn import ChempropBlock, EmbeddedChempropBlock, GraphEmbedding, Sum

    G = make_batch("qm9", 32, seed=3).collate("nodes").to(DEV)
    torch.manual_seed(3)
    enc = EmbeddedChempropBlock(GraphEmbedding(42, 13, 128), ChempropBlock(128, depth=3)).eval().to(DEV)
    fn = lambda G: Sum()(enc(G))  # noqa: E731
    with torch.no_grad():
        eager = fn(G).clone()
    assert torch.equal(GraphedForward(fn, G)(), eager)
