"""GPU: graph_loader (workers -> pinned batches or page-locked ring slots -> side-stream H2D) delivers device batches equal to
collate-then-.to(device), and the embedded encoder gives bit-identical outputs on them."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.mark.parametrize("pin_threads,ring_slots,background,feeder", [
    (0, 0, False, False), (3, 0, False, False), (0, 3, False, False), (0, 1, True, False), (0, 3, True, False),
    (2, 0, True, False), (0, 3, False, True), (0, 1, False, True), (0, 2, True, True)])
def test_graph_loader_batches_and_forward_bit_identical(pin_threads, ring_slots, background, feeder):
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
                              ring_slots=ring_slots, background=background, feeder=feeder):
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


def test_graph_feeder_epochs_early_stop_and_shuffle():
    """graph_loader over the DataLoader-free GraphFeeder (page-locked ring): two epochs, one of them
    abandoned after two batches, then a shuffled loader; every device batch equals the collate of
    the same molecules moved with .to(device)."""
    from notorch_amd.data.loader import graph_loader
    from notorch_amd.data.models.graph import BatchedGraph
    from notorch_amd.data.synth import make_batch

    graphs = make_batch("qm9", 300, seed=6).to_graphs()
    loader = graph_loader(graphs, 64, DEV, num_workers=3, ring_slots=2)
    assert loader.ring is not None
    for stop in (2, None):
        got = []
        for G in loader:
            assert loader.ring.registered  # page-locked after the workers forked (hipHostRegister)
            got.append(G)
            if stop is not None and len(got) == stop:
                break
        torch.cuda.synchronize()
        assert len(got) == (stop or 5)
        for i, G in enumerate(got):
            ref = BatchedGraph.from_graphs(graphs[64 * i:64 * (i + 1)]).to(DEV)
            for x, y in zip(G.tensors(), ref.tensors()):
                assert torch.equal(x, y)
    loader.batches.close()
    shuf = graph_loader(graphs, 64, DEV, num_workers=2, ring_slots=2, shuffle=True, drop_last=True,
                        generator=torch.Generator().manual_seed(3))
    perm = torch.randperm(300, generator=torch.Generator().manual_seed(3)).tolist()
    got = list(shuf)
    torch.cuda.synchronize()
    assert len(got) == 4
    for i, G in enumerate(got):
        ref = BatchedGraph.from_graphs([graphs[j] for j in perm[64 * i:64 * (i + 1)]]).to(DEV)
        for x, y in zip(G.tensors(), ref.tensors()):
            assert torch.equal(x, y)
    shuf.batches.close()
