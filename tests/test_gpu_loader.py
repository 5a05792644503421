"""GPU: graph_loader (workers -> pinned batches or page-locked ring slots -> side-stream H2D) delivers device batches equal to
collate-then-.to(device), and the embedded encoder gives bit-identical outputs on them."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.mark.parametrize("pin_threads,ring_slots", [(0, 0), (3, 0), (0, 3), (0, 1)])
def test_graph_loader_batches_and_forward_bit_identical(pin_threads, ring_slots):
    from notorch_amd.data.loader import graph_loader
    from notorch_amd.data.models.graph import BatchedGraph
    from notorch_amd.data.synth import make_batch
    from notorch_amd.nn import ChempropBlock, EmbeddedChempropBlock, GraphEmbedding, Sum

    graphs = make_batch("qm9", 256, seed=4).to_graphs()
    torch.manual_seed(0)
    enc = EmbeddedChempropBlock(GraphEmbedding(42, 13, 64), ChempropBlock(hidden_dim=64, depth=3)).eval().to(DEV)
    got = []
    with torch.no_grad():
        for G in graph_loader(graphs, 64, DEV, num_workers=2, pin_threads=pin_threads,
                              ring_slots=ring_slots):
            assert G.node_feats.device.type == "cuda" and G._nt_layout.dst_ptr.device.type == "cuda"
            got.append(Sum()(enc(G)))
    torch.cuda.synchronize()
    assert len(got) == 4
    # the batches arrive in the loader's order (several pin threads; ring slots reused, one slot per
    # worker: each batch waits for the previous one's copy to finish)
    with torch.no_grad():
        for i, r in enumerate(got):
            ref = Sum()(enc(BatchedGraph.from_graphs(graphs[64 * i:64 * (i + 1)]).to(DEV)))
            assert torch.equal(r, ref)
