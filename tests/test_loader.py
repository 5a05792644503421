"""CPU: the host feed (notorch_amd.data.loader) — DataLoader workers running the
native collate return exactly what BatchedGraph.from_graphs returns in the main process
(transforms/graph.py:45 -> graph.py:186-223), including the shipped CSR layout and tile plan."""
import pickle

import torch

from notorch_amd.data.loader import GraphCollator
from notorch_amd.data.models.graph import BatchedGraph
from notorch_amd.data.synth import make_batch


def _same(a, b):
    assert len(a) == len(b)
    for x, y in zip(a.tensors(), b.tensors()):
        assert x.dtype == y.dtype and torch.equal(x, y)
    la, lb = a._nt_layout, b._nt_layout
    assert la.deg_range == lb.deg_range and la.mol_max == lb.mol_max and la.type_range == lb.type_range
    assert la.plan[1] == lb.plan[1] and la.plan[3] == lb.plan[3]


def test_collator_in_workers_matches_main_process():
    graphs = make_batch("qm9", 96, seed=3).to_graphs()
    coll = GraphCollator("nodes")
    pickle.loads(pickle.dumps(coll))
    dl = torch.utils.data.DataLoader(graphs, batch_size=32, collate_fn=coll, num_workers=2)
    got = list(dl)
    assert len(got) == 3
    for i, G in enumerate(got):
        _same(G, BatchedGraph.from_graphs(graphs[32 * i:32 * (i + 1)], "nodes"))
        # the statistics still describe the unpickled tensors (no re-validation needed)
        assert G._layout_types_ok()


def test_graph_tensors_cover_layout():
    G = BatchedGraph.from_graphs(make_batch("qm9", 8, seed=1).to_graphs())
    ts = G.tensors()
    lay = G._nt_layout
    for t in (lay.dst_ptr, lay.dst_perm, lay.mol_ptr, lay.plan[0], lay.plan[2], G.batch_edge_index):
        assert any(t is u for u in ts)


def test_pack_one_buffer_same_values_and_pickles_as_one_storage():
    import io

    graphs = make_batch("qm9", 40, seed=5).to_graphs()
    ref = BatchedGraph.from_graphs(graphs, "nodes")
    G = BatchedGraph.from_graphs(graphs, "nodes").pack()
    _same(G, ref)
    buf = G._nt_packed
    assert G._packed_base() is buf
    assert {t.untyped_storage().data_ptr() for t in G.tensors()} == {buf.untyped_storage().data_ptr()}
    # through a worker queue (torch's shared-memory reductions): still one buffer in the main process
    dl = torch.utils.data.DataLoader(graphs, batch_size=40, collate_fn=GraphCollator("nodes"), num_workers=1)
    (G2,) = list(dl)
    _same(G2, ref)
    assert G2._packed_base() is not None
    # a graph whose features were replaced (update) falls back to per-tensor moves
    G3 = G.update(node_feats=G.node_feats.clone())
    assert G3._packed_base() is None
    G3.to("cpu")
    for x, y in zip(G3.tensors(), ref.tensors()):
        assert torch.equal(x, y)
    assert G3._nt_layout.type_range is None  # the statistics described the replaced tensor


def test_pinned_in_order_keeps_order_and_raises():
    """The prefetcher's pin pool (data/loader.py pinned_in_order): several threads, input order kept,
    a source error surfaces at its position, an early stop releases the feeder."""
    import random
    import time

    import pytest

    from notorch_amd.data.loader import pinned_in_order

    def slow(b):
        time.sleep(random.random() * 0.005)
        return b * 10

    assert list(pinned_in_order(range(40), 4, slow)) == [10 * i for i in range(40)]

    def src():
        yield 1
        yield 2
        raise ValueError("bad batch")

    got = []
    with pytest.raises(ValueError, match="bad batch"):
        for x in pinned_in_order(src(), 3, slow):
            got.append(x)
    assert got == [10, 20]

    def bad_pin(b):
        if b == 3:
            raise RuntimeError("pin failed")
        return b

    with pytest.raises(RuntimeError, match="pin failed"):
        list(pinned_in_order(range(10), 2, bad_pin))
    it = pinned_in_order(range(1000), 2, slow)
    assert next(it) == 0
    it.close()  # the feeder stops and the pool shuts down


def test_slot_ring_worker_batches_equal_main_process_collate():
    """Workers pack into SlotRing slots and ship only offsets (data/loader.py SlotBatch): the batch
    rebuilt over the ring equals from_graphs in the main process; slots are held until released; a
    batch larger than a slot takes the shared-memory path."""
    from notorch_amd.data.loader import SlotBatch, SlotRing

    graphs = make_batch("qm9", 96, seed=3).to_graphs()
    nbytes = BatchedGraph.from_graphs(graphs[:32]).packed_nbytes()
    ring = SlotRing(2, 3, nbytes * 3 // 2)
    dl = torch.utils.data.DataLoader(graphs, batch_size=32, collate_fn=GraphCollator("nodes", ring), num_workers=2)
    got = list(dl)
    assert all(isinstance(b, SlotBatch) for b in got)
    assert sorted(b.slot for b in got) == sorted({b.slot for b in got})  # distinct slots: none released yet
    assert ring.flags.sum().item() == 3
    for i, b in enumerate(got):
        G = b.load(ring)
        _same(G, BatchedGraph.from_graphs(graphs[32 * i:32 * (i + 1)], "nodes"))
        assert G._packed_base() is not None and G._layout_types_ok()
        base = ring.slot(b.slot).data_ptr()
        assert all(base <= t.data_ptr() < base + ring.slot_bytes for t in G.tensors())
        ring.release(b.slot)
    assert ring.flags.sum().item() == 0
    # slots too small: the ordinary shared-memory batch
    small = SlotRing(1, 2, 4096)
    (G,) = list(torch.utils.data.DataLoader(graphs[:32], batch_size=32, collate_fn=GraphCollator("nodes", small),
                                            num_workers=1))
    assert isinstance(G, BatchedGraph) and small.flags.sum().item() == 0
    _same(G, BatchedGraph.from_graphs(graphs[:32], "nodes"))
    # the collate outputs fit the slot but the plans do not: every tensor moved out, slot freed
    G0 = BatchedGraph.from_graphs(graphs[:32], "nodes")
    nine = [G0.node_feats, G0.edge_feats, G0.edge_index, G0.rev_index, G0.batch_node_index, G0.batch_edge_index,
            G0._nt_layout.dst_ptr, G0._nt_layout.dst_perm, G0._nt_layout.mol_ptr]
    tight = SlotRing(1, 1, sum((t.numel() * t.element_size() + 63) // 64 * 64 for t in nine) + 64)
    assert tight.slot_bytes < G0.packed_nbytes()
    (G,) = list(torch.utils.data.DataLoader(graphs[:32], batch_size=32, collate_fn=GraphCollator("nodes", tight),
                                            num_workers=1))
    assert isinstance(G, BatchedGraph) and tight.flags.sum().item() == 0
    _same(G, G0)
    # no free slot within the timeout: also the ordinary path
    ring.flags.fill_(1)
    assert ring.acquire(0, timeout_s=0.01) == -1
