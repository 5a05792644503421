"""Graph / BatchedGraph with the reference's field names and semantics, plus the device layout.

Mirrors ``notorch/data/models/graph.py`` (Graph :14-164, BatchedGraph :167-247) and
``notorch/utils/utils.py:34-40`` (``UpdateMixin.update``): same dataclass fields, ``num_nodes``,
``num_edges``, ``device``, ``.to``, ``len()`` and shallow-copy ``update``.

What is new is :class:`DeviceLayout`, the CSR view the kernels consume:

* ``dst_ptr[V+1]`` / ``dst_perm[E]`` (int32): in-edges of every node in ascending edge id
  (stable), i.e. the order in which the reference's CPU ``scatter_add_`` accumulates.
* ``mol_ptr[B+1]`` / ``mol_perm[V]`` (int32, ``mol_perm`` None when ``batch_node_index`` is
  sorted, which the collate guarantees): the nodes of every molecule, for the readouts.

``BatchedGraph.from_graphs`` (the collate, reference ``graph.py:186-223``) is vectorised and
builds that layout on the host, so it ships to the device with ``.to``.  A graph that arrives
without a layout (built by hand, or edited) gets one on the device via ``nt_csr_build``.

The reference collate offsets ``rev_index`` by the cumulative NODE count (``graph.py:200`` with
``:204``) instead of the cumulative edge count.  ``rev_offset="nodes"`` (default) reproduces that
bit for bit; ``rev_offset="edges"`` is the corrected collate.
"""
from __future__ import annotations

import ctypes
import os
import weakref
from itertools import repeat
from operator import attrgetter
from copy import copy
from dataclasses import InitVar, dataclass, field
from typing import Iterable, Literal, Optional

import numpy as np
import torch
from torch import Tensor

RevOffset = Literal["nodes", "edges"]


class UpdateMixin:
    """``notorch/utils/utils.py:34-40``: ``update`` returns a shallow copy (or self) with fields set."""

    def update(self, in_place: bool = False, **kwargs):
        other = self if in_place else copy(self)
        for key, val in kwargs.items():
            setattr(other, key, val)
        return other


@dataclass(eq=False)
class DeviceLayout:
    """CSR view of a (batched) graph consumed by the kernels.  All int32."""

    dst_ptr: Optional[Tensor] = None
    dst_perm: Optional[Tensor] = None
    mol_ptr: Optional[Tensor] = None
    mol_perm: Optional[Tensor] = None
    # identity of the tensors the layout was derived from (cache validity)
    edge_index: Optional[Tensor] = None
    batch_node_index: Optional[Tensor] = None
    validated: bool = False  # src/dst in [0,V), rev in [0,E) checked
    # fused-update tile plan (tile_ptr, ntiles, dst_sorted, zero_fill), derived lazily on the device
    # by notorch_amd.nn.gnn._engine.fused_plan; False = not available (in-degree > 32)
    plan: object = None
    # the fp32 layer kernel's wider plan: (tile_ptr, ntiles) of node-aligned tiles of <= 128 rows,
    # balanced over PLAN_NCU CUs (dst_sorted / zero_fill as in `plan`); False = not available
    plan_wide: object = None
    # backward CSRs (src -> nodes, rev_index -> edges), built lazily by _engine.backward_layout
    bwd: object = None
    # the fp32 layer kernel's row table (key, rev_index, E x 4 int32), built lazily by _engine.row_table
    row_table: object = None
    # the fused embedding init's type records (key, E x 4 int32), built lazily by _engine.embed_records
    embed_records: object = None
    # host-computed statistics the collate ships with the CSR, so a fresh batch needs no
    # device -> host sync: (max, min) in-degree, largest molecule, (min, max) type index of the
    # node / edge feature columns when they are integer type matrices
    deg_range: Optional[tuple] = None
    mol_max: Optional[int] = None
    type_range: Optional[tuple] = None
    # chunk plan of the dst CSR (hubs) and of the molecule CSR (large molecules): tensors or False
    dst_chunks: object = None
    mol_chunks: object = None
    type_src: object = None  # (weakref node_feats, weakref edge_feats) type_range was taken from
    # hub nodes of the dst CSR (in-degree > MAX_FUSED_IN_DEGREE): (hub ids int32, count, largest
    # non-hub in-degree), False when there are none; the fp32 fused plans then cut hubs at the stride
    hubs: object = None

    def __getstate__(self):
        # weak references do not pickle (DataLoader workers ship collated graphs): mark the type
        # statistics as describing the owning graph's features; Graph.__setstate__ re-binds them
        st = dict(self.__dict__)
        if st.get("type_src") is not None:
            st["type_src"] = "owner"
        return st

    def tensors(self) -> list:
        """Every tensor the layout owns (CSR arrays, plans, chunk plans)."""
        out = [t for t in (self.dst_ptr, self.dst_perm, self.mol_ptr, self.mol_perm) if t is not None]
        for p in (self.plan, self.plan_wide, self.dst_chunks, self.mol_chunks[1] if self.mol_chunks else None,
                  self.hubs):
            if p:
                out += [x for x in p if isinstance(x, Tensor)]
        return out

    def map_tensors(self, fn, edge_index: Tensor, batch_node_index: Optional[Tensor]) -> "DeviceLayout":
        """A copy of the layout with fn applied to every tensor it owns (device moves, pinning)."""
        mv = lambda t: None if t is None else fn(t)  # noqa: E731

        def mv_plan(p):  # (tensors and ints) tuples or False / None
            if not p:
                return p
            return tuple(fn(x) if isinstance(x, Tensor) else x for x in p)

        new = DeviceLayout(
            mv(self.dst_ptr),
            mv(self.dst_perm),
            mv(self.mol_ptr),
            mv(self.mol_perm),
            edge_index,
            batch_node_index,
            self.validated,
        )
        new.plan = mv_plan(self.plan)
        new.plan_wide = mv_plan(self.plan_wide)
        new.deg_range, new.mol_max, new.type_range = self.deg_range, self.mol_max, self.type_range
        new.dst_chunks = mv_plan(self.dst_chunks)
        new.hubs = mv_plan(self.hubs)
        if self.mol_chunks is not None and new.mol_ptr is not None:
            new.mol_chunks = (new.mol_ptr, mv_plan(self.mol_chunks[1]))
        return new

    def to(self, device, edge_index: Tensor, batch_node_index: Optional[Tensor]) -> "DeviceLayout":
        return self.map_tensors(lambda t: t.to(device, non_blocking=True), edge_index, batch_node_index)


def _rebaser(old: Tensor, new: Tensor):
    """Map a contiguous view into buffer ``old`` to the same bytes of buffer ``new``."""
    base = old.data_ptr()

    def fn(t: Tensor) -> Tensor:
        off = t.data_ptr() - base
        return new[off:off + t.numel() * t.element_size()].view(t.dtype).view(t.shape)

    return fn


@dataclass(repr=False, eq=False)
class Graph(UpdateMixin):
    """A single graph: ``node_feats`` V x *, ``edge_feats`` E x *, ``edge_index`` 2 x E,
    ``rev_index`` E (reference ``graph.py:14-39``)."""

    node_feats: Tensor
    edge_feats: Tensor
    edge_index: Tensor
    rev_index: Tensor
    device_: InitVar[object] = field(default=None, kw_only=True)

    def __post_init__(self, device_):
        self._device = device_
        self._nt_layout: Optional[DeviceLayout] = None
        self.to(device_)

    @property
    def num_nodes(self) -> int:
        return len(self.node_feats)

    @property
    def num_edges(self) -> int:
        return len(self.edge_feats)

    @property
    def device(self):
        return self._device

    def to(self, device, non_blocking: bool = False):
        """Move in place (reference graph.py:41-43).  non_blocking: asynchronous copies from pinned
        host memory (pin_memory()), ordered on the current stream.  A packed graph (pack()) moves
        as one buffer: one copy instead of one per tensor."""
        self._device = device
        if device is None:
            return self
        buf = self._packed_base()
        if buf is not None:
            new = buf.to(device, non_blocking=non_blocking)
            self._apply(_rebaser(buf, new), self)
            self._nt_packed = new
        else:
            self._apply(lambda t: t.to(device, non_blocking=non_blocking), self)
        return self

    def _apply(self, fn, other, types_ok: Optional[bool] = None) -> None:
        """other's fields and kernel layout := fn(self's); the layout's host statistics stay bound
        to the features when they described them (types_ok: that answer, taken before fn ran)."""
        if types_ok is None:
            types_ok = self._layout_types_ok()
        lay = getattr(self, "_nt_layout", None)
        for name in self._field_names():
            setattr(other, name, fn(getattr(self, name)))
        if lay is not None:
            moved = lay.map_tensors(fn, other.edge_index, getattr(other, "batch_node_index", None))
            if types_ok:
                moved.type_src = (weakref.ref(other.node_feats), weakref.ref(other.edge_feats),
                                  (other.node_feats._version, other.edge_feats._version))
            else:
                moved.type_range = None
            other._nt_layout = moved

    def _pack_plan(self):
        """(tensors, their byte offsets, total bytes) of pack()'s one-buffer layout, or None when a
        tensor is off the CPU or empty (the graph then stays unpacked)."""
        ts, seen = [], set()
        for t in self.tensors():
            if id(t) not in seen:
                seen.add(id(t))
                ts.append(t)
        if any(t.device.type != "cpu" or t.numel() == 0 for t in ts):
            return None
        offs, total = {}, 0
        for t in ts:
            offs[id(t)] = total
            total += (t.numel() * t.element_size() + 63) // 64 * 64
        return ts, offs, total

    def packed_nbytes(self) -> int:
        """Bytes of pack()'s buffer (0: the graph does not pack)."""
        plan = self._pack_plan()
        return 0 if plan is None else plan[2]

    def pack(self, shared: bool = False, out: Optional[Tensor] = None):
        """Copy every host tensor of the graph and its layout into ONE contiguous buffer (views at
        64-B aligned offsets), so pickling to the main process, pinning and the H2D copy each move
        one storage instead of ~15 (DataLoader workers: data/loader.py).  shared: allocate the
        buffer in shared memory, so that a worker's queue ships it without another copy.  out: a
        1-D uint8 CPU tensor of at least packed_nbytes() bytes to pack into (its first bytes)."""
        plan = self._pack_plan()
        if plan is None:
            return self
        ts, offs, total = plan
        # before any copy: with from_graphs(out=...) the fields are views of `out`, whose version
        # counter the copies below advance
        types_ok = self._layout_types_ok()
        if out is not None:
            if out.dtype != torch.uint8 or out.dim() != 1 or out.numel() < total or out.device.type != "cpu":
                raise ValueError(f"pack(out=...) needs a CPU uint8 vector of >= {total} bytes")
            buf = out[:total]
        elif shared:
            buf = torch.empty(0, dtype=torch.uint8).set_(torch.UntypedStorage._new_shared(total), 0, (total,), (1,))
        else:
            buf = torch.empty(total, dtype=torch.uint8)
        views = {}
        for t in ts:
            o = offs[id(t)]
            v = buf[o:o + t.numel() * t.element_size()].view(t.dtype).view(t.shape)
            if v.data_ptr() != t.data_ptr():  # from_graphs(out=...) already wrote it in place
                v.copy_(t)
            views[id(t)] = v
        self._apply(lambda t: views[id(t)], self, types_ok)
        self._nt_packed = buf
        return self

    def _packed_base(self) -> Optional[Tensor]:
        """The packed buffer if every tensor of the graph is still a contiguous view into it."""
        buf = getattr(self, "_nt_packed", None)
        if buf is None:
            return None
        lo, hi = buf.data_ptr(), buf.data_ptr() + buf.numel()
        for t in self.tensors():
            p = t.data_ptr()
            if t.device != buf.device or not t.is_contiguous() or p < lo or p + t.numel() * t.element_size() > hi:
                return None
        return buf

    def _feature_tensors(self) -> list:
        return [self.node_feats, self.edge_feats, self.edge_index, self.rev_index]

    def tensors(self) -> list:
        """Every tensor of the graph and of its kernel layout."""
        lay = getattr(self, "_nt_layout", None)
        return self._feature_tensors() + (lay.tensors() if lay is not None else [])

    def pin_memory(self):
        """Copy of the graph with every host tensor (features, indices, CSR layout, plans) in pinned
        memory, so .to(device, non_blocking=True) is an asynchronous DMA.  torch's DataLoader calls
        this on collated batches when pin_memory=True."""
        other = copy(self)
        buf = self._packed_base()
        if buf is not None:
            # the packed buffer's copy through ctypes.memmove, which releases the GIL (Tensor.pin_memory
            # holds it for the whole copy: 7 MB at config 2, stalling the thread that launches kernels)
            new = torch.empty(buf.numel(), dtype=torch.uint8, pin_memory=True)
            ctypes.memmove(new.data_ptr(), buf.data_ptr(), buf.numel())
            self._apply(_rebaser(buf, new), other)
            other._nt_packed = new
        else:
            self._apply(Tensor.pin_memory, other)
            other._nt_packed = None
        return other

    def _field_names(self) -> list:
        return ["node_feats", "edge_feats", "edge_index", "rev_index"]

    def __setstate__(self, state):
        self.__dict__.update(state)
        lay = state.get("_nt_layout")
        if lay is not None and lay.type_src == "owner":
            lay.type_src = (weakref.ref(self.node_feats), weakref.ref(self.edge_feats),
                            (self.node_feats._version, self.edge_feats._version))

    def _layout_types_ok(self) -> bool:
        lay = getattr(self, "_nt_layout", None)
        return lay is not None and lay.type_range is not None and _same_types(lay, self.node_feats, self.edge_feats)

    @property
    def A(self) -> Tensor:
        """Dense adjacency matrix (reference ``graph.py:55-64``)."""
        src, dest = self.edge_index.unbind(0)
        A = torch.zeros(self.num_nodes, self.num_nodes)
        A[src, dest] = 1
        return A

    @property
    def P(self) -> Tensor:
        """Markov transition matrix (reference ``graph.py:66-72``)."""
        A = self.A
        return A / A.sum(1, keepdim=True)

    @property
    def dense2sparse(self) -> Tensor:
        """V x V map from a dense (u, v) pair to its edge id, -1 if absent (``graph.py:74-94``)."""
        src, dest = self.edge_index.unbind(0)
        index = -torch.ones(self.num_nodes, self.num_nodes, dtype=torch.long)
        index[src, dest] = torch.arange(self.edge_index.shape[1])
        return index

    def __repr__(self) -> str:
        return (
            f"{type(self).__name__}(node_feats: Tensor(shape={tuple(self.node_feats.shape)}), "
            f"edge_feats: Tensor(shape={tuple(self.edge_feats.shape)}), device={self._device})"
        )


@dataclass(repr=False, eq=False, kw_only=True)
class BatchedGraph(Graph):
    """A batch of graphs (reference ``graph.py:167-247``)."""

    batch_node_index: Tensor
    batch_edge_index: Tensor
    size: InitVar[Optional[int]] = None

    def __post_init__(self, device_, size):
        super().__post_init__(device_)
        # reference graph.py:184 stores a 0-d tensor when size is None (len() then fails);
        # we store an int either way.
        self._size = int(self.batch_node_index.max()) + 1 if size is None else int(size)

    def __len__(self) -> int:
        return self._size

    def _field_names(self) -> list:
        return ["node_feats", "edge_feats", "edge_index", "rev_index", "batch_node_index", "batch_edge_index"]

    def _feature_tensors(self) -> list:
        return [getattr(self, n) for n in self._field_names()]

    @classmethod
    def from_graphs(cls, Gs: Iterable[Graph], rev_offset: RevOffset = "nodes", *,
                    out: Optional[Tensor] = None) -> "BatchedGraph":
        """Collate (reference ``graph.py:186-223``) + the CSR layout the kernels consume.

        ``rev_offset="nodes"`` reproduces the reference exactly, including the offset of
        ``rev_index`` by the cumulative node count (``graph.py:200``); ``"edges"`` fixes it.
        Host graphs go through the native one-pass collate (``nt_collate_graphs``: copies, offsets,
        validation and an O(V+E) counting-sort CSR in C++); graphs already on a device are
        collated with device ops.  out (host graphs; data/loader.py): a 1-D uint8 CPU buffer the
        native collate writes its outputs into, at the offsets pack() gives them, so that a later
        pack(out=out) copies only the layout's plans (the outputs may be views into out).
        """
        Gs = list(Gs)
        if len(Gs) == 0:
            raise ValueError("from_graphs needs at least one graph")
        if rev_offset not in ("nodes", "edges"):
            raise ValueError(f"rev_offset must be 'nodes' or 'edges', got {rev_offset!r}")
        fast = _collate_py()
        r = fast.graph_arrays(Gs) if fast is not None else (1,)
        if r[0] != 1 or (all(map(attrgetter("edge_index.is_cpu"), Gs)) and all(map(attrgetter("node_feats.is_cpu"), Gs))):
            return _native_collate(cls, Gs, rev_offset, r, out)
        return cls._from_graphs_device(Gs, rev_offset)

    @classmethod
    def _from_graphs_device(cls, Gs: list, rev_offset: RevOffset) -> "BatchedGraph":
        """Vectorised torch collate (graphs on a device)."""
        n_nodes = torch.tensor([len(G.node_feats) for G in Gs], dtype=torch.long)
        n_edges = torch.tensor([len(G.edge_feats) for G in Gs], dtype=torch.long)
        node_off = torch.cumsum(n_nodes, 0) - n_nodes
        edge_off = torch.cumsum(n_edges, 0) - n_edges
        B = len(Gs)
        graph_ids = torch.arange(B)
        node_feats = torch.cat([G.node_feats for G in Gs], dim=0)
        edge_feats = torch.cat([G.edge_feats for G in Gs], dim=0)
        n_ei = torch.tensor([G.edge_index.shape[-1] for G in Gs], dtype=torch.long)
        n_rev = torch.tensor([len(G.rev_index) for G in Gs], dtype=torch.long)
        edge_index = torch.cat([G.edge_index.reshape(2, -1).long() for G in Gs], dim=1)
        edge_index = edge_index + torch.repeat_interleave(node_off, n_ei).unsqueeze(0)
        rev_base = node_off if rev_offset == "nodes" else edge_off
        rev_index = torch.cat([G.rev_index.long() for G in Gs], dim=0)
        rev_index = rev_index + torch.repeat_interleave(rev_base, n_rev)
        batch_node_index = torch.repeat_interleave(graph_ids, n_nodes)
        batch_edge_index = torch.repeat_interleave(graph_ids, n_edges)
        BG = cls(
            node_feats,
            edge_feats,
            edge_index,
            rev_index,
            device_=None,
            batch_node_index=batch_node_index,
            batch_edge_index=batch_edge_index,
            size=B,
        )
        BG._nt_layout = host_layout(edge_index, rev_index, len(node_feats), batch_node_index, B,
                                    node_feats, edge_feats)
        if Gs[-1].device is not None:  # reference passes device_=G.device of the last graph
            BG.to(Gs[-1].device)
        return BG

    def __repr__(self) -> str:
        return super().__repr__()[:-1] + f", batch_size={len(self)})"


def _row_bytes(x: Tensor) -> int:
    """Bytes of one row (dim 0) of x, also when x has no rows."""
    return int(np.prod(x.shape[1:], dtype=np.int64)) * x.element_size()


_COLLATE_PY: list = []


def _collate_py():
    """The collate's CPython helper (notorch_amd/lib/_collate_py*.so, built by make), or None."""
    if not _COLLATE_PY:
        import glob
        import importlib.util

        mod = None
        lib_dir = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "lib")
        for path in glob.glob(os.path.join(lib_dir, "_collate_py*.so")):
            spec = importlib.util.spec_from_file_location("_collate_py", path)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            break
        _COLLATE_PY.append(mod)
    return _COLLATE_PY[0]


def _native_collate(cls, Gs: list, rev_offset: RevOffset, r: tuple, out: Optional[Tensor] = None) -> "BatchedGraph":
    """BatchedGraph.from_graphs through nt_collate_graphs (host C++; see include/notorch_amd.h).
    r: _collate_py().graph_arrays(Gs), or (1,) for the Python walk."""
    B = len(Gs)
    i64 = torch.int64

    def _c(x):  # contiguous int64 view, without a call per graph in the common case
        return x if (x.dtype is i64 and x.is_contiguous()) else x.to(i64).contiguous()

    T = Tensor
    if r[0] == 2:
        raise RuntimeError("from_graphs: node_feats of the graphs differ in dtype or row shape")
    if r[0] == 3:
        raise RuntimeError("from_graphs: edge_feats of the graphs differ in dtype or row shape")
    if r[0] == 4:
        raise RuntimeError("from_graphs: edge_index / rev_index do not match edge_feats")
    if r[0] == 0:  # the per-graph walk in C++ (csrc/host/collate_py.cpp)
        _, n_nodes, n_edges, gptr, V, E = r
        nd, ed = Gs[0].node_feats, Gs[0].edge_feats
        return _collate_into(cls, Gs, rev_offset, n_nodes, n_edges, V, E, nd, ed,
                             [gptr[k].numpy() for k in range(4)], out)
    # per-graph work through C-level map() over the tensors' own methods (the extension's fallback:
    # non-contiguous features, non-int64 indices)
    nf = list(map(attrgetter("node_feats"), Gs))
    ef = list(map(attrgetter("edge_feats"), Gs))
    ei = list(map(attrgetter("edge_index"), Gs))
    rv = list(map(attrgetter("rev_index"), Gs))
    if not all(map(T.is_contiguous, nf)):
        nf = [x.contiguous() for x in nf]
    if not all(map(T.is_contiguous, ef)):
        ef = [y.contiguous() for y in ef]
    if not (all(map(T.is_contiguous, ei)) and {z.dtype for z in ei} == {i64}):
        ei = [_c(z) for z in ei]
    if not (all(map(T.is_contiguous, rv)) and {r.dtype for r in rv} == {i64}):
        rv = [_c(r) for r in rv]
    nn_ = list(map(T.size, nf, repeat(0)))  # Tensor.size(0): C-level (len() goes through Python)
    ne_ = list(map(T.size, ef, repeat(0)))
    nd, ed = nf[0], ef[0]
    if len({(x.dtype, x.shape[1:]) for x in nf}) != 1:
        raise RuntimeError("from_graphs: node_feats of the graphs differ in dtype or row shape")
    if len({(x.dtype, x.shape[1:]) for x in ef}) != 1:
        raise RuntimeError("from_graphs: edge_feats of the graphs differ in dtype or row shape")
    if list(map(T.numel, ei)) != [2 * n for n in ne_] or list(map(T.numel, rv)) != ne_:
        raise RuntimeError("from_graphs: edge_index / rev_index do not match edge_feats")
    n_nodes = torch.tensor(nn_, dtype=i64)
    n_edges = torch.tensor(ne_, dtype=i64)
    V, E = int(n_nodes.sum()), int(n_edges.sum())

    def ptrs(ts):  # the B data pointers as one array
        return np.fromiter(map(T.data_ptr, ts), dtype=np.uint64, count=B)

    return _collate_into(cls, Gs, rev_offset, n_nodes, n_edges, V, E, nd, ed, [ptrs(nf), ptrs(ef), ptrs(ei), ptrs(rv)],
                         out)


def _collate_into(cls, Gs, rev_offset, n_nodes, n_edges, V, E, nd, ed, gptrs, out=None) -> "BatchedGraph":
    """nt_collate_graphs over the graphs' data pointers (gptrs: four arrays of B pointers: node_feats,
    edge_feats, edge_index, rev_index), then the layout's host statistics and plans.  out: write the
    nine collate outputs into this uint8 buffer at pack()'s offsets (when they fit)."""
    from notorch_amd import _lib

    B = len(Gs)
    specs = [((V,) + tuple(nd.shape[1:]), nd.dtype), ((E,) + tuple(ed.shape[1:]), ed.dtype), ((2, E), torch.int64),
             ((E,), torch.int64), ((V,), torch.int64), ((E,), torch.int64), ((V + 1,), torch.int32),
             ((E,), torch.int32), ((B + 1,), torch.int32)]
    sizes = [int(np.prod(sh, dtype=np.int64)) * torch.empty(0, dtype=dt).element_size() for sh, dt in specs]
    if out is not None and min(sizes) > 0 and sum((n + 63) // 64 * 64 for n in sizes) <= out.numel():
        outs, o = [], 0  # pack()'s layout: the graph's fields, then dst_ptr, dst_perm, mol_ptr, 64-B aligned
        for (sh, dt), n in zip(specs, sizes):
            outs.append(out[o:o + n].view(dt).view(sh))
            o += (n + 63) // 64 * 64
    else:
        outs = [torch.empty(sh, dtype=dt) for sh, dt in specs]
    node_out, edge_out, edge_index, rev_index, bni, bei, dst_ptr, dst_perm, mol_ptr = outs
    gp = [np.ascontiguousarray(a) for a in gptrs]
    lib = _lib.load()
    _lib.check(lib.nt_collate_graphs(
        B, gp[0].ctypes.data, n_nodes.data_ptr(), _row_bytes(nd),
        gp[1].ctypes.data, n_edges.data_ptr(), _row_bytes(ed),
        gp[2].ctypes.data, gp[3].ctypes.data, 0 if rev_offset == "nodes" else 1, node_out.data_ptr(), edge_out.data_ptr(),
        edge_index.data_ptr(), rev_index.data_ptr(), bni.data_ptr(), bei.data_ptr(),
        dst_ptr.data_ptr(), dst_perm.data_ptr(), mol_ptr.data_ptr(),
    ))
    BG = cls(node_out, edge_out, edge_index, rev_index, device_=None, batch_node_index=bni,
             batch_edge_index=bei, size=B)
    lay = DeviceLayout(dst_ptr, dst_perm, edge_index=edge_index, validated=True)
    # rev_offset="nodes" can push rev_index past E only for graphs with fewer edges than nodes
    # (reference quirk): leave such batches to the device-side check
    lay.validated = E == 0 or int(rev_index.numpy().max()) < E  # numpy: no intra-op pool wake-up
    lay.mol_ptr, lay.mol_perm, lay.batch_node_index = mol_ptr, None, bni
    host_stats(lay, dst_ptr.numpy(), E, mol_ptr.numpy(), node_out, edge_out)
    BG._nt_layout = lay
    if Gs[-1].device is not None:  # reference passes device_=G.device of the last graph
        BG.to(Gs[-1].device)
    return BG


def host_layout(
    edge_index: Tensor,
    rev_index: Tensor,
    num_nodes: int,
    batch_node_index: Optional[Tensor] = None,
    num_graphs: Optional[int] = None,
    node_feats: Optional[Tensor] = None,
    edge_feats: Optional[Tensor] = None,
) -> DeviceLayout:
    """Build the CSR layout on the host (numpy stable argsort == ascending edge id per node)."""
    ei = edge_index.detach().cpu().numpy()
    E = ei.shape[1]
    src, dst = ei[0], ei[1]
    rev = rev_index.detach().cpu().numpy()
    validated = bool(
        E == 0
        or (
            src.min() >= 0
            and src.max() < num_nodes
            and dst.min() >= 0
            and dst.max() < num_nodes
            and rev.min() >= 0
            and rev.max() < E
        )
    )
    if not validated:
        # leave the layout to the device path, which raises IndexError like the reference's gather
        return None  # type: ignore[return-value]
    dst_perm = np.argsort(dst, kind="stable").astype(np.int32)
    counts = np.bincount(dst, minlength=num_nodes)
    dst_ptr = np.zeros(num_nodes + 1, dtype=np.int32)
    np.cumsum(counts, out=dst_ptr[1:])
    lay = DeviceLayout(
        torch.from_numpy(dst_ptr),
        torch.from_numpy(dst_perm),
        edge_index=edge_index,
        validated=True,
    )
    if batch_node_index is not None and num_graphs is not None:
        b = batch_node_index.detach().cpu().numpy()
        if b.size == 0 or (b.min() >= 0 and b.max() < num_graphs):
            mol_ptr = np.zeros(num_graphs + 1, dtype=np.int32)
            np.cumsum(np.bincount(b, minlength=num_graphs), out=mol_ptr[1:])
            sorted_ = b.size < 2 or bool(np.all(b[1:] >= b[:-1]))
            lay.mol_ptr = torch.from_numpy(mol_ptr)
            lay.mol_perm = None if sorted_ else torch.from_numpy(np.argsort(b, kind="stable").astype(np.int32))
            lay.batch_node_index = batch_node_index
    host_stats(lay, dst_ptr, E, None if lay.mol_ptr is None else lay.mol_ptr.numpy(), node_feats, edge_feats)
    return lay


# ---- host-side plans (numpy restatements of the device planners; same arrays, no device sync) ----
MAX_FUSED_IN_DEGREE = 32  # nt_dmpnn_tile_plan's limit; a graph with larger in-degrees has hubs
# hub graphs: nodes with more than HUB_CUT_DEGREE in-edges are cut at the stride by nt_dmpnn_tile_plan_hubs
# and aggregated by nt_dmpnn_hub_aggregate (fp32; bf16 takes the unfused path), so the rest of the plan
# keeps node-aligned tiles of in-degree <= 9 (8 scan rounds) instead of 32
HUB_CUT_DEGREE = 9
LONG_SEGMENT = 64  # segments longer than this aggregate through the chunked reduce
CHUNK_ROWS = 32  # rows per chunk of nt_segment_reduce_chunked


PLAN_NCU = 256  # kernels.PLAN_NCU: the CU count the balanced plans are cut for
PLAN_SLOTS64 = PLAN_NCU  # kernels.PLAN_SLOTS64 (64-row plans)
WIDE_TILE_ROWS = 128  # rows of the diagnostic build's update_fk_kernel tiles (the shipping kernels: 64)


def host_tile_stride(E: int, max_in_degree: int, rows: int, ncu: int) -> int:
    """nt_dmpnn_tile_stride restated: tiles of at most `rows` rows, balanced to whole rounds of ncu."""
    if E <= 0 or rows < 1 or max_in_degree > rows:
        return 0
    lmax = rows + 1 - max(int(max_in_degree), 1)
    if ncu <= 0:
        return lmax
    rounds = (E + ncu * lmax - 1) // (ncu * lmax)
    L = (E + rounds * ncu - 1) // (rounds * ncu)
    return max(1, min(L, lmax))


def check_tile_rows(tile_ptr: np.ndarray, rows: int) -> None:
    """The layer kernels hold at most `rows` rows per tile: a plan with a larger tile is rejected where
    it is built (the kernels keep no device status word to report it later)."""
    if len(tile_ptr) > 1:
        mx = int(np.diff(tile_ptr.astype(np.int64)).max())
        if mx > rows:
            raise ValueError(f"tile plan holds a tile of {mx} rows > the kernel's {rows}: the max in-degree "
                             "given to the planner is below the graph's")


def host_tile_ptr(dst_ptr: np.ndarray, E: int, stride: int, hub_degree: int = 0, rows: Optional[int] = None) -> tuple:
    """(tile_ptr[ntiles+1], ntiles) as nt_dmpnn_tile_plan builds them: tile k starts at
    dst_ptr[first v with dst_ptr[v] >= k stride]; with hub_degree > 0 as nt_dmpnn_tile_plan_hubs
    (a target inside a node with more in-edges is kept as the cut).  rows: checked tile capacity."""
    ntiles = (E + stride - 1) // stride if E > 0 else 0
    tile_ptr = np.empty(ntiles + 1, dtype=np.int32)
    if ntiles:
        t = np.arange(ntiles, dtype=np.int64) * stride
        if hub_degree > 0:
            v = np.searchsorted(dst_ptr, t, side="right") - 1  # the node holding position t
            b, e = dst_ptr[v].astype(np.int64), dst_ptr[v + 1].astype(np.int64)
            tile_ptr[:ntiles] = np.where((b == t) | (e - b > hub_degree), t, e)
        else:
            v = np.searchsorted(dst_ptr, t, side="left")
            tile_ptr[:ntiles] = dst_ptr[v]
    tile_ptr[ntiles] = E
    if rows is not None:
        check_tile_rows(tile_ptr, rows)
    return torch.from_numpy(tile_ptr), ntiles


def host_tile_plan(dst_ptr: np.ndarray, E: int, max_in_degree: int, rows: int = 64, ncu: int = 0,
                   hub_degree: int = 0, dsts: Optional[Tensor] = None):
    """(tile_ptr[ntiles+1], ntiles, dst_sorted[E]) exactly as nt_dmpnn_tile_plan (hub_degree > 0:
    nt_dmpnn_tile_plan_hubs) builds them with the stride of nt_dmpnn_tile_stride(E, max_in_degree,
    rows, ncu)."""
    stride = host_tile_stride(E, max_in_degree, rows, ncu) if E > 0 else 1
    tile_ptr, ntiles = host_tile_ptr(dst_ptr, E, stride, hub_degree, rows)
    return tile_ptr, ntiles, _segment_ids(dst_ptr)[0] if dsts is None else dsts


def _segment_ids(seg_ptr: np.ndarray) -> tuple:
    """(ids int32 tensor: position -> segment, max count, min count) of a CSR offset array: one C++ pass
    through the collate helper when it is built and seg_ptr is int32, else numpy."""
    fast = _collate_py()
    if fast is not None and seg_ptr.dtype == np.int32 and seg_ptr.flags.c_contiguous:
        r = fast.segment_ids(torch.from_numpy(seg_ptr))
        if r is not None:
            return r
    counts = np.diff(seg_ptr.astype(np.int64))
    ids = np.repeat(np.arange(len(counts), dtype=np.int32), counts)
    return torch.from_numpy(ids), (int(counts.max()) if counts.size else 0), (int(counts.min()) if counts.size else 0)


def _minmax(X: Tensor) -> Optional[tuple]:
    """(min, max) of a CPU int64 tensor (None when empty; numpy's vectorised reductions)."""
    if X.numel() == 0:
        return None
    xn = X.numpy()
    return int(xn.min()), int(xn.max())


def host_chunk_plan(seg_ptr: np.ndarray, chunk: int = CHUNK_ROWS):
    """(chunk_pos[nchunks+1], nchunks, chunk_ptr[nseg+1], chunk_seg[nchunks], comb_seg[ncomb]) exactly
    as kernels.chunk_plan builds them."""
    sp = seg_ptr.astype(np.int64)
    n = sp[1:] - sp[:-1]
    nch = (n + chunk - 1) // chunk
    chunk_ptr = np.zeros(len(n) + 1, dtype=np.int64)
    np.cumsum(nch, out=chunk_ptr[1:])
    nchunks = int(chunk_ptr[-1])
    seg_of = np.repeat(np.arange(len(n)), nch)
    k_in_seg = np.arange(nchunks) - chunk_ptr[seg_of]
    chunk_pos = np.empty(nchunks + 1, dtype=np.int32)
    chunk_pos[:nchunks] = sp[seg_of] + k_in_seg * chunk
    chunk_pos[nchunks] = seg_ptr[-1]
    multi = nch != 1
    chunk_seg = np.where(multi[seg_of], -1, seg_of).astype(np.int32)
    comb_seg = np.nonzero(multi)[0].astype(np.int32)
    return (torch.from_numpy(chunk_pos), nchunks, torch.from_numpy(chunk_ptr.astype(np.int32)),
            torch.from_numpy(chunk_seg), torch.from_numpy(comb_seg))


def host_stats(lay: DeviceLayout, dst_ptr: np.ndarray, E: int, mol_ptr: Optional[np.ndarray],
               node_feats: Optional[Tensor] = None, edge_feats: Optional[Tensor] = None) -> None:
    """Fill the layout's host statistics and plans from the host CSR (one O(V + E) pass)."""
    V = len(dst_ptr) - 1
    dsts, dmax, dmin = _segment_ids(dst_ptr)  # dst node of every dst-sorted position, degree range
    lay.deg_range = (dmax, dmin) if V > 0 else (0, 0)
    maxdeg, mindeg = lay.deg_range
    hub = 0
    lay.hubs = False
    if E > 0 and V > 0 and maxdeg > MAX_FUSED_IN_DEGREE:  # hubs: cut at the stride (fp32 plans)
        deg = np.diff(dst_ptr.astype(np.int64))
        is_hub = deg > HUB_CUT_DEGREE
        ids = np.nonzero(is_hub)[0].astype(np.int32)
        rest = deg[~is_hub]
        lay.hubs = (torch.from_numpy(ids), int(ids.size), int(rest.max()) if rest.size else 0)
        hub, maxdeg = HUB_CUT_DEGREE, lay.hubs[2]
    if E > 0 and V > 0:
        tile_ptr, ntiles, dsts = host_tile_plan(dst_ptr, E, maxdeg, rows=64, ncu=PLAN_SLOTS64, hub_degree=hub,
                                                dsts=dsts)
        lay.plan = (tile_ptr, ntiles, dsts, mindeg == 0)
        lay.plan_wide = host_tile_ptr(dst_ptr, E, host_tile_stride(E, maxdeg, WIDE_TILE_ROWS, PLAN_NCU), hub,
                                      WIDE_TILE_ROWS)
    lay.dst_chunks = host_chunk_plan(dst_ptr) if lay.deg_range[0] > LONG_SEGMENT else False
    if mol_ptr is not None:
        n = np.diff(mol_ptr.astype(np.int64))
        lay.mol_max = int(n.max()) if n.size else 0
        if lay.mol_ptr is not None:
            lay.mol_chunks = (lay.mol_ptr, host_chunk_plan(mol_ptr) if lay.mol_max > LONG_SEGMENT else False)
    if node_feats is not None and edge_feats is not None:
        lay.type_src = (weakref.ref(node_feats), weakref.ref(edge_feats), (node_feats._version, edge_feats._version))
    tr = []
    for X in (node_feats, edge_feats):
        if X is not None and X.dim() == 2 and X.dtype == torch.int64 and X.device.type == "cpu":
            r = _minmax(X)
            tr.append(r if r is not None else (0, -1))
        else:
            tr.append(None)
    lay.type_range = tuple(tr)


def _same_types(lay: DeviceLayout, node_feats: Tensor, edge_feats: Tensor) -> bool:
    """Whether lay.type_range describes exactly these feature tensors (same objects, unmodified)."""
    src = lay.type_src
    if not isinstance(src, tuple):
        return False
    return src[0]() is node_feats and src[1]() is edge_feats and src[2] == (node_feats._version, edge_feats._version)


def types_in_range(lay: Optional[DeviceLayout], node_types: Tensor, edge_types: Tensor, num_node_types: int,
                   num_edge_types: int) -> Optional[bool]:
    """Host answer to "are all type indices inside the tables?" from the collate's statistics:
    True / False, or None when the layout carries no statistics for these tensors."""
    if lay is None or lay.type_range is None or not _same_types(lay, node_types, edge_types):
        return None
    (n0, n1), (e0, e1) = lay.type_range
    return n0 >= 0 and n1 < num_node_types and e0 >= 0 and e1 < num_edge_types
