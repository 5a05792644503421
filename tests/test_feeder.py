"""CPU: GraphFeeder (data/feeder.py), the DataLoader-free host feed: forked workers collate batches
straight into shared-memory ring slots in batch order; the batches equal BatchedGraph.from_graphs
(reference notorch/data/models/graph.py:186-223) of the same molecules, across epochs, early stops,
shuffling, spills and worker errors."""
import pytest
import torch

from notorch_amd.data.feeder import GraphFeeder
from notorch_amd.data.loader import SlotBatch
from notorch_amd.data.models.graph import BatchedGraph, Graph
from notorch_amd.data.synth import make_batch


def _same(a, b):
    assert len(a) == len(b)
    for x, y in zip(a.tensors(), b.tensors()):
        assert x.dtype == y.dtype and torch.equal(x, y)
    la, lb = a._nt_layout, b._nt_layout
    assert (la.deg_range, la.mol_max, la.type_range) == (lb.deg_range, lb.mol_max, lb.type_range)


def _host(f, item):
    if isinstance(item, SlotBatch):
        G = item.load(f.ring)
        G._apply(lambda t: t.clone(), G)  # every tensor off the slot before it is released
        f.ring.release(item.slot)
        return G
    return item


def test_feeder_batches_epochs_and_early_stop():
    graphs = make_batch("qm9", 230, seed=3).to_graphs()
    f = GraphFeeder(graphs, 32, num_workers=3, slots_per_worker=2)
    try:
        assert len(f) == 8
        for epoch in range(2):
            got = [_host(f, x) for x in f]
            assert len(got) == 8
            for i, G in enumerate(got):
                _same(G, BatchedGraph.from_graphs(graphs[32 * i:32 * (i + 1)]))
        # an epoch abandoned after two batches, then a full one
        it = iter(f)
        for _ in range(2):
            _host(f, next(it))
        del it
        got = [_host(f, x) for x in f]
        assert len(got) == 8
        _same(got[7], BatchedGraph.from_graphs(graphs[224:]))
    finally:
        f.close()


def test_feeder_shuffle_drop_last_and_spill():
    graphs = make_batch("zinc", 50, seed=4).to_graphs()
    g = torch.Generator().manual_seed(7)
    f = GraphFeeder(graphs, 16, num_workers=2, shuffle=True, drop_last=True, generator=g, slot_bytes=4096)
    try:
        perm = torch.randperm(50, generator=torch.Generator().manual_seed(7)).tolist()
        got = [_host(f, x) for x in f]  # 4096-byte slots: every batch spills through the pipe
        assert len(got) == 3 and all(isinstance(G, BatchedGraph) for G in got)
        for i, G in enumerate(got):
            _same(G, BatchedGraph.from_graphs([graphs[j] for j in perm[16 * i:16 * (i + 1)]]))
    finally:
        f.close()


def test_feeder_worker_error_is_raised():
    graphs = make_batch("qm9", 40, seed=5).to_graphs()
    bad = Graph(graphs[0].node_feats, graphs[0].edge_feats, graphs[0].edge_index.clone(), graphs[0].rev_index)
    bad.edge_index[1, 0] = 999  # out of range: the native collate rejects it
    f = GraphFeeder(graphs[:20] + [bad] + graphs[20:], 10, num_workers=2)
    try:
        with pytest.raises(RuntimeError, match="batch 2"):
            for x in f:
                _host(f, x)
        # the feeder still works for the next epoch of a good dataset view
    finally:
        f.close()
    with pytest.raises(ValueError):
        GraphFeeder(graphs, 0)
