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
