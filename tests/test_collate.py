"""CPU: the collate (native nt_collate_graphs for host graphs, vectorised torch on a device) is bit-identical to the restated reference collate
(notorch/data/models/graph.py:186-223) in both rev-offset modes, and its CSR layout is exact."""
import numpy as np
import pytest
import torch

from notorch_amd.data.models.graph import BatchedGraph, Graph
from notorch_amd.data.synth import make_batch
from oracle import collate_ref

FIELDS = ["node_feats", "edge_feats", "edge_index", "rev_index", "batch_node_index", "batch_edge_index"]


@pytest.mark.parametrize("kind,n", [("qm9", 64), ("zinc", 16), ("polymer", 2)])
@pytest.mark.parametrize("mode", ["nodes", "edges"])
def test_from_graphs_bit_identical(kind, n, mode):
    batch = make_batch(kind, n, seed=3)
    Gs = batch.to_graphs()
    ref = collate_ref.from_graphs(Gs, rev_offset=mode)
    for BG in (BatchedGraph.from_graphs(Gs, rev_offset=mode), batch.collate(mode)):
        for f in FIELDS:
            assert torch.equal(getattr(BG, f), ref[f]), f
        assert len(BG) == ref["size"]


def test_reference_rev_offset_quirk_reproduced():
    """graph.py:200 offsets rev_index by the node count: in a multi-molecule batch most rev entries
    do NOT point at the reverse edge; the fixed collate makes rev == e ^ 1."""
    G = make_batch("qm9", 256, seed=0).collate("nodes")
    e = torch.arange(G.num_edges)
    assert (G.rev_index != (e ^ 1)).float().mean() > 0.9
    Gf = make_batch("qm9", 256, seed=0).collate("edges")
    assert torch.equal(Gf.rev_index, e ^ 1)


def test_layout_csr_exact():
    G = make_batch("qm9", 128, seed=1).collate("nodes")
    lay = G._nt_layout
    dst = G.edge_index[1].numpy()
    assert np.array_equal(lay.dst_perm.numpy(), np.argsort(dst, kind="stable"))
    assert np.array_equal(lay.dst_ptr.numpy()[1:], np.cumsum(np.bincount(dst, minlength=G.num_nodes)))
    assert lay.mol_perm is None  # batch_node_index sorted
    assert np.array_equal(np.diff(lay.mol_ptr.numpy()), np.bincount(G.batch_node_index.numpy()))


def test_edge_cases_zero_bond_molecule_and_empty():
    # a single-atom molecule with no bonds (the reference MolToGraph would crash, quirk 2)
    one = Graph(torch.tensor([[1, 12, 20, 25, 30, 36, 41]]), torch.zeros(0, 2, dtype=torch.long),
                torch.zeros(2, 0, dtype=torch.long), torch.zeros(0, dtype=torch.long))
    Gs = make_batch("qm9", 3, seed=2).to_graphs()
    mixed = [Gs[0], one, Gs[1]]
    BG = BatchedGraph.from_graphs(mixed)
    ref = collate_ref.from_graphs(mixed)
    for f in FIELDS:
        assert torch.equal(getattr(BG, f), ref[f]), f
    with pytest.raises(ValueError):
        BatchedGraph.from_graphs([])


def test_layout_travels_with_to_and_update():
    G = make_batch("qm9", 8, seed=4).collate("nodes")
    lay = G._nt_layout
    G2 = G.update(node_feats=torch.zeros(G.num_nodes, 3))
    assert G2._nt_layout is lay  # shallow copy shares the layout
    G3 = G.to("cpu")
    assert G3._nt_layout.edge_index is G3.edge_index


def test_collate_is_picklable():
    import pickle

    G = make_batch("qm9", 4, seed=5).collate("nodes")
    G2 = pickle.loads(pickle.dumps(G))
    assert torch.equal(G2.edge_index, G.edge_index) and len(G2) == 4
    from notorch_amd.data.models.graph import types_in_range

    # the shipped statistics still describe the unpickled features (DataLoader workers)
    assert types_in_range(G2._nt_layout, G2.node_feats, G2.edge_feats, 42, 13) is True
    assert G2._nt_layout.plan[1] == G._nt_layout.plan[1]


def test_native_collate_matches_device_path_and_layout():
    """nt_collate_graphs (host C++) == the vectorised torch collate, field for field, and its
    counting-sort CSR == a stable argsort."""
    Gs = make_batch("zinc", 48, seed=6).to_graphs()
    for mode in ("nodes", "edges"):
        BG = BatchedGraph.from_graphs(Gs, rev_offset=mode)
        TG = BatchedGraph._from_graphs_device(Gs, mode)
        for f in FIELDS:
            assert torch.equal(getattr(BG, f), getattr(TG, f)), f
        lay = BG._nt_layout
        dst = BG.edge_index[1].numpy()
        assert np.array_equal(lay.dst_perm.numpy(), np.argsort(dst, kind="stable"))
        assert np.array_equal(lay.mol_ptr.numpy(), TG._nt_layout.mol_ptr.numpy())


def test_native_collate_float_features_and_errors():
    from notorch_amd._lib import NativeLibraryError

    Gs = make_batch("qm9", 5, seed=7).to_graphs()
    Fs = [Graph(torch.randn(G.num_nodes, 3), torch.randn(G.num_edges, 5, dtype=torch.float64),
                G.edge_index, G.rev_index) for G in Gs]
    BG = BatchedGraph.from_graphs(Fs)
    assert torch.equal(BG.node_feats, torch.cat([G.node_feats for G in Fs]))
    assert torch.equal(BG.edge_feats, torch.cat([G.edge_feats for G in Fs]))
    bad = Graph(Gs[0].node_feats, Gs[0].edge_feats, Gs[0].edge_index.clone(), Gs[0].rev_index)
    bad.edge_index[1, 0] = Gs[0].num_nodes  # one past the molecule's atoms
    with pytest.raises(NativeLibraryError, match="out of range"):
        BatchedGraph.from_graphs([Gs[1], bad])
    mixed = [Gs[0], Graph(Gs[1].node_feats.float(), Gs[1].edge_feats, Gs[1].edge_index, Gs[1].rev_index)]
    with pytest.raises(RuntimeError, match="differ"):
        BatchedGraph.from_graphs(mixed)


def test_host_plans_ship_with_the_collate():
    """The collate ships the statistics and plans a fresh batch needs (no device -> host sync):
    in-degree range, tile plan (tiles cut at node boundaries, <= 64 rows, every node's in-edges in
    one tile), chunk plans for hubs, molecule size, type-index ranges."""
    import numpy as np

    from notorch_amd.data.models.graph import BatchedGraph, types_in_range
    from notorch_amd.data.synth import make_batch

    b = make_batch("qm9", 300, seed=4)
    for G in (b.collate("nodes"), BatchedGraph.from_graphs(b.to_graphs(), rev_offset="edges")):
        lay = G._nt_layout
        dst_ptr = lay.dst_ptr.numpy().astype(np.int64)
        deg = np.diff(dst_ptr)
        assert lay.deg_range == (deg.max(), deg.min())
        tile_ptr, ntiles, dsts, zero_fill = lay.plan
        tp = tile_ptr.numpy()
        assert tp[0] == 0 and tp[-1] == G.num_edges and len(tp) == ntiles + 1
        assert (np.diff(tp) <= 64).all() and (np.diff(tp) >= 0).all()
        assert np.isin(tp, dst_ptr).all()  # cuts only at node boundaries
        assert (dsts.numpy() == np.repeat(np.arange(G.num_nodes), deg)).all()
        assert zero_fill == (deg.min() == 0)
        assert lay.dst_chunks is False
        assert lay.mol_max == int(np.bincount(G.batch_node_index.numpy()).max())
        assert types_in_range(lay, G.node_feats, G.edge_feats, 42, 13) is True
        assert types_in_range(lay, G.node_feats, G.edge_feats, 41, 13) is False
        G.node_feats[0, 0] = 5  # in-place edit: the statistics no longer describe the tensor
        assert types_in_range(lay, G.node_feats, G.edge_feats, 42, 13) is None
    P = make_batch("polymer", 2, seed=1).collate("nodes")
    lay = P._nt_layout
    assert lay.deg_range[0] > 32
    # hubs (in-degree > 32): listed, and the plans cut them at the stride while every other cut
    # stays on a node boundary; tiles within the row capacity of the non-hub in-degree
    dst_ptr = lay.dst_ptr.numpy().astype(np.int64)
    deg = np.diff(dst_ptr)
    ids, nhub, rest = lay.hubs
    assert ids.dtype == torch.int32 and nhub == ids.numel() > 0
    from notorch_amd.data.models.graph import HUB_CUT_DEGREE

    assert (ids.numpy() == np.nonzero(deg > HUB_CUT_DEGREE)[0]).all() and rest == deg[deg <= HUB_CUT_DEGREE].max()
    hub_pos = np.zeros(P.num_edges + 1, dtype=bool)
    for v in ids.numpy():
        hub_pos[dst_ptr[v] + 1:dst_ptr[v + 1]] = True  # interior positions of a hub's in-edge range
    starts = set(dst_ptr.tolist())
    for (tile_ptr, ntiles), rows in ((lay.plan[:2], 64), (lay.plan_wide, 128)):
        tp = tile_ptr.numpy().astype(np.int64)
        assert tp[0] == 0 and tp[-1] == P.num_edges and len(tp) == ntiles + 1
        assert np.diff(tp).max() <= rows and np.diff(tp).min() >= 0
        assert all(int(t) in starts or hub_pos[t] for t in tp)
        assert hub_pos[tp].any()  # some cut falls inside a hub
    chunk_pos, nchunks, chunk_ptr, chunk_seg, comb_seg = lay.dst_chunks
    assert chunk_pos.numel() == nchunks + 1 and int(chunk_ptr[-1]) == nchunks
    assert (np.diff(chunk_pos.numpy()) <= 32).all()
    nch = np.diff(chunk_ptr.numpy())
    single = np.nonzero(nch == 1)[0]
    assert np.array_equal(chunk_seg.numpy()[chunk_ptr.numpy()[single]], single)
    assert (chunk_seg.numpy() >= 0).sum() == single.size
    assert np.array_equal(comb_seg.numpy(), np.nonzero(nch != 1)[0])


def test_all_zero_bond_batch_collates():
    """Every molecule without a bond (E = 0 in the whole batch): the native collate still returns
    the reference layout (empty edge tensors of the right shapes, one molecule per node)."""
    import torch

    from notorch_amd.data.models.graph import BatchedGraph, Graph

    one = Graph(torch.tensor([[1, 12, 20, 25, 30, 36, 41]]), torch.zeros(0, 2, dtype=torch.long),
                torch.zeros(2, 0, dtype=torch.long), torch.zeros(0, dtype=torch.long))
    G = BatchedGraph.from_graphs([one, one, one])
    assert G.num_nodes == 3 and G.num_edges == 0 and len(G) == 3
    assert G.edge_feats.shape == (0, 2) and G.edge_index.shape == (2, 0) and G.rev_index.shape == (0,)
    assert G.batch_node_index.tolist() == [0, 1, 2]
    assert G._nt_layout.dst_ptr.tolist() == [0, 0, 0, 0]


def test_host_tile_stride_matches_library():
    """The host restatement of nt_dmpnn_tile_stride (collate-shipped plans) equals the library's."""
    from notorch_amd import _lib
    from notorch_amd.data.models.graph import host_tile_stride

    lib = _lib.load()
    for E in (1, 7, 614, 77_628, 620_000, 2_370_000):
        for maxdeg in (1, 4, 13, 32):
            for rows, ncu in ((64, 0), (128, 256), (128, 0), (64, 256), (128, 80)):
                assert host_tile_stride(E, maxdeg, rows, ncu) == lib.nt_dmpnn_tile_stride(E, maxdeg, rows, ncu)


def test_collate_ships_balanced_plans():
    """The collate's plans: the 64-row plan (bf16 layer kernel, and update_fk_kernel's 64-row variants)
    and the 128-row plan of the shipping fp32 update_fk_kernel, node-aligned, cut to whole rounds of
    256 tiles (config 2: about 5 and 3 tiles per CU)."""
    import numpy as np

    from notorch_amd.data.synth import make_batch

    G = make_batch("qm9", 4096, seed=1000).collate("nodes")
    lay = G._nt_layout
    starts = set(lay.dst_ptr.numpy().tolist())
    for (tile_ptr, ntiles), rows, rounds in ((lay.plan[:2], 64, 5), (lay.plan_wide, 128, 3)):
        tp = tile_ptr.numpy().astype(np.int64)
        sizes = np.diff(tp)
        assert tp[0] == 0 and tp[-1] == G.num_edges and sizes.max() <= rows and sizes.min() > 0
        assert all(int(t) in starts for t in tp)  # every cut is a node boundary
        assert (rounds - 1) * 256 < ntiles <= rounds * 256, (rows, ntiles)
    assert lay.plan[1] > lay.plan_wide[1]  # the 64-row plan has more, smaller tiles


def test_collate_helper_walk_matches_python_walk():
    """csrc/host/collate_py.cpp (the per-graph walk in C++) feeds nt_collate_graphs exactly what the
    Python walk does: same batch, same layout; non-contiguous features and int32 indices take the
    Python walk; mismatched rows / index sizes raise the same errors."""
    from notorch_amd.data.models import graph as gm

    fast = gm._collate_py()
    assert fast is not None, "notorch_amd/lib/_collate_py*.so not built (run make)"
    Gs = make_batch("zinc", 40, seed=11).to_graphs()
    r = fast.graph_arrays(Gs)
    assert r[0] == 0 and r[4] == sum(G.num_nodes for G in Gs) and r[5] == sum(G.num_edges for G in Gs)
    assert r[3][0, 3].item() == Gs[3].node_feats.data_ptr() and r[3][3, 5].item() == Gs[5].rev_index.data_ptr()
    for mode in ("nodes", "edges"):
        a = gm._native_collate(BatchedGraph, Gs, mode, r)
        b = gm._native_collate(BatchedGraph, Gs, mode, (1,))
        for f in FIELDS:
            assert torch.equal(getattr(a, f), getattr(b, f)), f
        la, lb = a._nt_layout, b._nt_layout
        for x, y in zip(la.tensors(), lb.tensors()):
            assert torch.equal(x, y)
        assert (la.deg_range, la.mol_max, la.type_range) == (lb.deg_range, lb.mol_max, lb.type_range)
    # Python-walk cases: non-contiguous features, int32 indices
    nc = [Graph(G.node_feats.t().contiguous().t(), G.edge_feats, G.edge_index, G.rev_index) for G in Gs[:4]]
    i32 = [Graph(G.node_feats, G.edge_feats, G.edge_index.int(), G.rev_index.int()) for G in Gs[:4]]
    for case in (nc, i32):
        assert fast.graph_arrays(case) == (1,)
        BG = BatchedGraph.from_graphs(case)
        ref = collate_ref.from_graphs(case)
        for f in FIELDS:
            assert torch.equal(getattr(BG, f), ref[f].to(getattr(BG, f).dtype)), f
    # errors
    g0 = Gs[0]
    bad_nf = [g0, Graph(g0.node_feats[:, :3].contiguous(), g0.edge_feats, g0.edge_index, g0.rev_index)]
    bad_ef = [g0, Graph(g0.node_feats, g0.edge_feats.float(), g0.edge_index, g0.rev_index)]
    bad_ix = [g0, Graph(g0.node_feats, g0.edge_feats, g0.edge_index, g0.rev_index[:-1])]
    for case, code, msg in ((bad_nf, 2, "node_feats"), (bad_ef, 3, "edge_feats"), (bad_ix, 4, "rev_index")):
        assert fast.graph_arrays(case) == (code,)
        with pytest.raises(RuntimeError, match=msg):
            BatchedGraph.from_graphs(case)
    with pytest.raises(TypeError):
        fast.graph_arrays(3)


def test_segment_ids_helper_matches_numpy():
    """The collate helper's segment_ids (dst-sorted node ids + degree range, graph.py host_stats) equals
    numpy's repeat / diff, with empty segments, an empty pointer and a non-monotone pointer (None)."""
    import numpy as np

    from notorch_amd.data.models import graph as gm

    fast = gm._collate_py()
    if fast is None:
        pytest.skip("collate helper not built")
    rng = np.random.default_rng(5)
    for counts in (rng.integers(0, 5, 1000), np.zeros(7, dtype=np.int64), np.array([3]), np.array([], dtype=np.int64)):
        sp = np.zeros(len(counts) + 1, dtype=np.int32)
        np.cumsum(counts, out=sp[1:])
        ids, mx, mn = fast.segment_ids(torch.from_numpy(sp))
        assert ids.dtype == torch.int32
        assert np.array_equal(ids.numpy(), np.repeat(np.arange(len(counts), dtype=np.int32), counts))
        assert (mx, mn) == ((int(counts.max()), int(counts.min())) if len(counts) else (0, 0))
    assert fast.segment_ids(torch.tensor([0, 3, 2], dtype=torch.int32)) is None
    ids, mx, mn = gm._segment_ids(np.array([0, 2, 2, 5], dtype=np.int32))
    assert ids.tolist() == [0, 0, 2, 2, 2] and (mx, mn) == (3, 0)


def test_collate_helper_reads_fields_without_an_instance_dict():
    """graph_arrays reads dataclass fields from the instance dict; objects whose fields are slots or
    properties (duck-typed reference graphs) take the generic attribute lookup with the same result."""
    from notorch_amd.data.models import graph as gm

    fast = gm._collate_py()
    if fast is None:
        pytest.skip("collate helper not built")

    class Slotted:
        __slots__ = ("node_feats", "edge_feats", "edge_index", "rev_index")

        def __init__(self, G):
            self.node_feats, self.edge_feats, self.edge_index, self.rev_index = (
                G.node_feats, G.edge_feats, G.edge_index, G.rev_index)

    class Props:
        def __init__(self, G):
            self._g = G

        node_feats = property(lambda self: self._g.node_feats)
        edge_feats = property(lambda self: self._g.edge_feats)
        edge_index = property(lambda self: self._g.edge_index)
        rev_index = property(lambda self: self._g.rev_index)

    Gs = make_batch("qm9", 12, seed=13).to_graphs()
    ref = fast.graph_arrays(Gs)
    for wrap in (Slotted, Props):
        r = fast.graph_arrays([wrap(G) for G in Gs])
        assert r[0] == 0 and r[4:] == ref[4:]
        for x, y in zip(r[1:4], ref[1:4]):
            assert torch.equal(x, y)

    class Missing:
        node_feats = edge_feats = edge_index = None

    assert fast.graph_arrays([Missing()]) == (1,)
