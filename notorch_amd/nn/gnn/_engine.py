"""Device engine behind ChempropBlock / readouts: layout management, the fused layer loop and the
autograd wrapper.

Forward (per call, all on ``torch.cuda.current_stream()``, inputs already resident).  Fused path
(every node's in-degree <= 32 and h % 4 == 0 — molecules; hub graphs cut their hubs into sub-runs):

    nt_dmpnn_init         H0 = Xv[src] + Xe  fused with  S = scatter(act(H0), dst)  chemprop.py:82-83,37-39
      (GraphEmbedding models: nt_dmpnn_init_embed from the type indices, over the graph's type records)
    for l in 0..d-1:
      nt_dmpnn_update_fused  H_{l+1} = H_l + W_l (S[src] - act(H_l)[rev]) + b_l      chemprop.py:40-41, residual.py:28
                             S = scatter(act(H_{l+1}), dst)   (last layer: node = scatter(H_d, dst),
                                                               chemprop.py:86)

d + 1 launches (+ one nt_dmpnn_pack_weights_fk launch pair per new set of weights).  Otherwise
(dropout, or no fused plan):

    nt_dmpnn_init; for l: nt_dmpnn_update, nt_segment_reduce; nt_segment_reduce (node)   2 + 2d launches

bf16 features (BASELINE config 3) run the same d + 1 launch sequence on the bf16 kernels
(csrc/bf16.hip: the 64-edge-tile update fused with the next aggregation).  Activations without a
kernel code, or layers that differ in activation / dropout, run layer by layer
(block_forward_layerwise).

Backward (training): the forward keeps (H_l, S_l) of every layer; per layer,
last to first (csrc/backward.hip, csrc/wgrad.hip):

    nt_dmpnn_weight_grad_fk  dW_l = G^T A_l, db_l = colsum(G), A_l = S_l[src] - act(H_l)[rev] formed
                             while staging (fp32 h <= 320: the two-part fp16 split; above it
                             nt_dmpnn_weight_grad's bf16x6; bf16: the bf16 weight-grad kernel)
    nt_dmpnn_update_fused    dA = G W_l and dS = scatter_sum(dA, src) in ONE launch of the layer kernel
                             over the src-sorted plan (dA_plan; nt_dmpnn_dense_matmul + nt_segment_reduce
                             where the plan does not apply; bf16: the bf16 layer kernel's dense mode)
    nt_dmpnn_edge_backward   G <- G + act'(H_l) * (dS[dst] / c - scatter_sum(dA, rev))  (rev CSR)
      (max / min: nt_segment_arg + nt_dmpnn_edge_backward_arg, fp32 and bf16: dS[dst] reaches only the arg)

then dXe = G, dXv = scatter_sum(G, src).
"""
from __future__ import annotations

import os
import threading
import weakref
from typing import Optional, Sequence

import torch
from torch import Tensor

from notorch_amd import _lib
from notorch_amd import kernels as K
from notorch_amd._lib import NT_ACT_IDENTITY
from notorch_amd.data.models.graph import DeviceLayout

_IDENTITY = (NT_ACT_IDENTITY, 0.0)
_RELU = (_lib.NT_ACT_RELU, 0.0)
# backward: dA and dS = sum_src dA in one fused launch (dA_plan); NT_FUSED_DA=0 keeps dense_matmul +
# segment_reduce (A/B)
_FUSED_DA = os.environ.get("NT_FUSED_DA", "1") != "0"
# fp32 weight gradient: "kernel" (nt_dmpnn_weight_grad_fk for h <= 320, else nt_dmpnn_weight_grad),
# "kernel6" (nt_dmpnn_weight_grad, bf16x6) or "library" (message + split-K library GEMM)
_WGRAD_DEFAULT = "kernel"

# Optional per-launch timer for the dominant kernel (bench.py sets it): a list that receives
# (start, end) torch.cuda.Event pairs recorded on the launch stream around every nt_dmpnn_update.
UPDATE_EVENTS: Optional[list] = None
# What the last layer-update launch ran (bench.py's roofline): kernel, numerics, padded MFMA shape.
LAST_UPDATE_INFO: dict = {}


def _note_update(kind: str, dtype: torch.dtype, h: int, rows: int = 0) -> None:
    """Record which layer kernel the forward ran (bench labels): the variant is the library's own
    report of its last launch (nt_last_kernel), so the label cannot drift from the dispatch."""
    kp, np_ = 32 * ((h + 31) // 32), 16 * ((h + 15) // 16)
    launched = _lib.load().nt_last_kernel().decode()
    short = launched.split(" ")[0].rstrip(":") or "update"
    if dtype == torch.bfloat16:
        info = dict(numerics="bf16 storage, bf16 MFMA, fp32 accumulate", products=1)
    elif short in ("update_fk_kernel", "update_fw_kernel"):
        info = dict(numerics="fp32 via scaled two-part fp16 split (3 fp16 MFMA products, fp32 accumulate)",
                    products=3)
    else:
        info = dict(numerics="exact fp32 MFMA", products=1)
    tail = {"fused": "aggregation of the next layer fused",
            "persistent": "no tile plan: hub graph, aggregation by the chunked segment reduce"}.get(kind, "unfused")
    info.update(kernel=f"{launched} ({tail})", kernel_short=short.replace("_kernel", ""),
                fused=kind == "fused", kpad=kp, npad=np_, rows=rows)
    LAST_UPDATE_INFO.clear()
    LAST_UPDATE_INFO.update(info)


# ------------------------------------------------------------------------------------ layouts
def _validate_indices(edge_index: Tensor, rev_index: Tensor, V: int) -> None:
    E = edge_index.shape[-1]
    if rev_index.numel() != E:
        raise RuntimeError(f"rev_index has {rev_index.numel()} entries for {E} edges")
    if E == 0:
        return
    mm = torch.stack(
        [edge_index.min(), edge_index.max(), rev_index.min(), rev_index.max()]
    ).cpu()  # one sync per new graph (the collate path validates on the host instead)
    if mm[0] < 0 or mm[1] >= V:
        raise IndexError(f"edge_index out of range for {V} nodes")
    if mm[2] < 0 or mm[3] >= E:
        raise IndexError(f"rev_index out of range for {E} edges")


def dst_layout(G) -> DeviceLayout:
    """The in-edge CSR of ``G`` on its device: cached from the collate, else built with nt_csr_build."""
    ei = G.edge_index
    lay: Optional[DeviceLayout] = getattr(G, "_nt_layout", None)
    if (
        lay is not None
        and lay.dst_ptr is not None
        and lay.validated
        and lay.edge_index is ei
        and lay.dst_ptr.device == ei.device
    ):
        return lay
    V = G.node_feats.shape[0]
    _validate_indices(ei, G.rev_index, V)
    dst = ei[1].contiguous()
    dst_ptr, dst_perm = K.csr_build(dst, V, check_bounds=False)
    new = DeviceLayout(dst_ptr, dst_perm, edge_index=ei, validated=True)
    if lay is not None and lay.mol_ptr is not None and lay.mol_ptr.device == ei.device:
        new.mol_ptr, new.mol_perm, new.batch_node_index = lay.mol_ptr, lay.mol_perm, lay.batch_node_index
    try:
        G._nt_layout = new
    except AttributeError:  # a foreign graph object that refuses new attributes: no caching
        pass
    return new


def mol_layout(G) -> tuple[Tensor, Optional[Tensor]]:
    """(mol_ptr, mol_perm) of a BatchedGraph: nodes of every molecule, for the readouts."""
    bni = G.batch_node_index
    B = len(G)
    lay: Optional[DeviceLayout] = getattr(G, "_nt_layout", None)
    if (
        lay is not None
        and lay.mol_ptr is not None
        and lay.batch_node_index is bni
        and lay.mol_ptr.device == bni.device
        and lay.mol_ptr.numel() == B + 1
    ):
        return lay.mol_ptr, lay.mol_perm
    mol_ptr, mol_perm = K.csr_build(bni.contiguous(), B, check_bounds=True)
    if lay is None:
        lay = DeviceLayout()
    lay.mol_ptr, lay.mol_perm, lay.batch_node_index = mol_ptr, mol_perm, bni
    try:
        G._nt_layout = lay
    except AttributeError:
        pass
    return mol_ptr, mol_perm


LONG_SEGMENT = 64  # segments longer than this switch the aggregation to the chunked reduce


def _degree_range(lay: DeviceLayout) -> tuple[int, int]:
    """(max, min) in-degree of the layout's dst CSR; one host sync per layout, cached."""
    mm = getattr(lay, "deg_range", None)
    if mm is None:
        deg = lay.dst_ptr[1:] - lay.dst_ptr[:-1]
        if deg.numel() == 0:
            mm = (0, 0)
        else:
            t = torch.stack([deg.max(), deg.min()]).cpu()
            mm = (int(t[0]), int(t[1]))
        lay.deg_range = mm
    return mm


MAX_FUSED_IN_DEGREE = 32  # larger in-degrees do not fit node-aligned tiles: the graph has hubs
# the hub-graph init (nt_dmpnn_init with skip_degree = MAX_FUSED_IN_DEGREE, then the chunked init over
# the skipped nodes' chunks) needs every multi-chunk segment to be a skipped node (notorch_amd.h)
assert K.CHUNK_ROWS >= MAX_FUSED_IN_DEGREE, "chunk rows must cover the wave init's in-degree cut"
HUB_DEGREE = 9  # in a hub graph, nodes with more in-edges are cut at the stride and reduced separately


def hub_info(lay: DeviceLayout):
    """(hub ids int32, count, largest non-hub in-degree) of the dst CSR when some node has more than
    MAX_FUSED_IN_DEGREE in-edges (hubs: every node with more than HUB_DEGREE), else None.  Cached on
    the layout (the host collate ships it); one sync otherwise."""
    if lay.hubs is None:
        hubs = False
        if lay.dst_ptr.numel() > 1 and _degree_range(lay)[0] > MAX_FUSED_IN_DEGREE:
            deg = lay.dst_ptr[1:] - lay.dst_ptr[:-1]
            is_hub = deg > HUB_DEGREE
            ids = torch.nonzero(is_hub).view(-1).to(torch.int32)
            rest = int(torch.where(is_hub, torch.zeros_like(deg), deg).max())
            hubs = (ids, ids.numel(), rest)
        lay.hubs = hubs
    return lay.hubs or None


def zero_rows_needed(lay: DeviceLayout, src: Tensor, V: int) -> tuple[bool, bool, bool]:
    """Which node-row outputs need a zero fill because no row of a plan writes them: (out, mid, bwd) =
    some node has in-degree 0 (the final node output: torch_scatter's empty segment is 0), some node
    has in-degree 0 and out-degree > 0 (an intermediate S row that a later S[src] gather reads), some
    node has out-degree 0 and in-degree > 0 (a dS row that the edge backward's dS[dst] reads).  Bond
    graphs have in-degree = out-degree, so only `out` can hold (isolated atoms).  Cached; the first
    call syncs once unless the in-degrees alone decide it."""
    key = (src.data_ptr(), src.numel(), V)
    hit = getattr(lay, "zero_rows", None)
    if hit is None or hit[0] != key:
        zf_out = V > 0 and _degree_range(lay)[1] == 0
        mid = bwd = False
        if zf_out or (V > 0 and src.numel() > 0):
            indeg = (lay.dst_ptr[1:] - lay.dst_ptr[:-1])
            outdeg = torch.bincount(src, minlength=V)[:V]
            t = torch.stack([((indeg == 0) & (outdeg > 0)).any(), ((outdeg == 0) & (indeg > 0)).any()]).cpu()
            mid, bwd = bool(t[0]), bool(t[1])
        hit = (key, (zf_out, mid, bwd))
        lay.zero_rows = hit
    return hit[1]


def fused_plan(lay: DeviceLayout, V: int, E: int, rows: int = 64, dtype: torch.dtype = torch.float32):
    """Tile plan of the fused update for this layout with tiles of at most ``rows`` (64 or 128) rows,
    balanced to whole rounds over PLAN_NCU CUs, as (tile_ptr, ntiles, dst_sorted, zero_fill), cached on
    it.  Hub nodes (more than HUB_DEGREE in-edges, polymer graphs) are cut at the stride; the fp32
    layer leaves their aggregation to nt_dmpnn_hub_aggregate (None for bf16: those graphs take the
    unfused path).  One sync per layout."""
    hubs = hub_info(lay) if E > 0 and V > 0 else None
    if hubs is not None and dtype != torch.float32:
        return None
    hub, maxdeg = (HUB_DEGREE, hubs[2]) if hubs is not None else (0, None)
    if lay.plan is None:
        plan = False
        if E > 0 and V > 0:
            mx, mindeg = _degree_range(lay)
            tile_ptr, ntiles, dsts = K.tile_plan(lay.dst_ptr, E, mx if maxdeg is None else maxdeg, rows=64,
                                                 ncu=K.PLAN_SLOTS64, hub_degree=hub)
            plan = (tile_ptr, ntiles, dsts, mindeg == 0)
        lay.plan = plan
    if not lay.plan:
        return None
    if rows <= 64:
        return lay.plan
    if lay.plan_wide is None:  # node-aligned tiles of <= 128 rows, balanced over the CUs
        mx = _degree_range(lay)[0] if maxdeg is None else maxdeg
        tile_ptr, ntiles, _ = K.tile_plan(lay.dst_ptr, E, mx, rows=128, ncu=K.PLAN_NCU, hub_degree=hub)
        lay.plan_wide = (tile_ptr, ntiles)
    return lay.plan_wide[0], lay.plan_wide[1], lay.plan[2], lay.plan[3]


def fused_max_in_degree(lay: DeviceLayout) -> int:
    """The in-degree the fused kernel's segmented scan must cover: the largest non-hub in-degree."""
    hubs = hub_info(lay)
    return _degree_range(lay)[0] if hubs is None else hubs[2]


def dst_chunks(lay: DeviceLayout):
    """Chunk plan of the dst CSR when some node's in-degree exceeds LONG_SEGMENT (hubs), else None."""
    ch = getattr(lay, "dst_chunks", None)
    if ch is None:
        ch = False
        if lay.dst_ptr.numel() > 1 and _degree_range(lay)[0] > LONG_SEGMENT:
            ch = K.chunk_plan(lay.dst_ptr)
        lay.dst_chunks = ch
    return ch or None


def hub_chunk_ids(lay: DeviceLayout, chunks) -> Tensor:
    """The chunks of the dst chunk plan that belong to segments longer than MAX_FUSED_IN_DEGREE (the
    hubs' part of a hub graph's init), int32, cached on the layout with the plan; one sync."""
    hit = getattr(lay, "hub_chunk_ids", None)
    if hit is None or hit[0] is not chunks[0]:
        chunk_ptr = chunks[2].long()
        nch = chunk_ptr[1:] - chunk_ptr[:-1]
        deg = (lay.dst_ptr[1:] - lay.dst_ptr[:-1]).long()
        seg_of = torch.repeat_interleave(torch.arange(deg.numel(), device=deg.device), nch, output_size=chunks[1])
        ids = torch.nonzero(deg[seg_of] > MAX_FUSED_IN_DEGREE).flatten().to(torch.int32)
        hit = (chunks[0], ids)
        lay.hub_chunk_ids = hit
    return hit[1]


def _aggregate(X, seg_ptr, perm, nseg, reduce, act, chunks, out=None, amax=None):
    """scatter(act(X), seg) by the chunked reduce (skewed segments) or the plain one; amax (fp32,
    1 device float) is raised to max|out| (fused into the chunked reduce, a separate pass otherwise)."""
    if chunks is not None:
        return K.segment_reduce_chunked(X, seg_ptr, perm, nseg, chunks, reduce=reduce, act=act, out=out,
                                        amax=amax)
    out = K.segment_reduce(X, seg_ptr, perm, nseg, reduce=reduce, act=act, out=out)
    if amax is not None:
        K.absmax(out, amax)
    return out


def _fused_enabled() -> bool:
    return os.environ.get("NT_FUSED", "1") != "0"


# ------------------------------------------------------------------------------------ forward
# Packed-weight cache: the MFMA fragment image of a parameter is re-derived only when the
# parameter changes (torch bumps Tensor._version on every in-place update, e.g. optimizer.step(),
# and a new storage changes data_ptr), so inference forwards reuse it and training forwards
# repack after every step.
# (Keyed by id() with a weakref check: tensors cannot be WeakKeyDictionary keys because their
# __eq__ is element-wise.)
_PACKED: dict[int, tuple] = {}


def _multi_packable(W: Tensor) -> bool:
    """fp32 weights whose image is the fk image alone (shipping library, h % 4 == 0): packed in one
    launch pair for all layers (nt_dmpnn_pack_weights_fk), with the backward's W^T image alongside."""
    return (W.dtype == torch.float32 and W.dim() == 2 and W.shape[0] % 4 == 0 and W.is_contiguous()
            and not _lib.DIAG)


def pack_layer_weights(weights: Sequence[Tensor], with_t: bool = False) -> list[Tensor]:
    """One packed MFMA image per layer; shared layers (same tensor) are packed once.  with_t (a
    training forward, fp32): the images of W^T too (packed_transpose), from the same launch pair."""
    out: list = [None] * len(weights)
    stale = []  # (index, W) needing a pack
    for i, W in enumerate(weights):
        key = (W.data_ptr(), W._version, tuple(W.shape), W.device)
        hit = _PACKED.get(id(W))
        if hit is None or hit[0]() is not W or hit[1] != key or (with_t and hit[3] is None):
            stale.append((i, W))
        else:
            out[i] = hit[2]
    multi = [(i, W) for i, W in stale if _multi_packable(W)]
    uniq: dict = {}
    for i, W in multi:
        uniq.setdefault(id(W), W)
    groups: dict = {}
    for W in uniq.values():
        groups.setdefault((W.shape[0], W.device), []).append(W)
    for ws in groups.values():
        for c in range(0, len(ws), 16):
            chunk = ws[c:c + 16]
            imgs, imgsT = K.pack_weights_fk_multi([W.detach() for W in chunk], with_t=with_t)
            for j, W in enumerate(chunk):
                _remember(W, imgs[j], None if imgsT is None else imgsT[j])
    for i, W in stale:
        if not _multi_packable(W):
            _remember(W, K.pack_weights(W.detach()), None)
        out[i] = _PACKED[id(W)][2]
    return out


def _remember(W: Tensor, Wp: Tensor, WpT: Optional[Tensor]) -> None:
    key = (W.data_ptr(), W._version, tuple(W.shape), W.device)
    wid = id(W)
    ref = weakref.ref(W, lambda _r, wid=wid: _PACKED.pop(wid, None))
    _PACKED[wid] = (ref, key, Wp, WpT)


def packed_transpose(W: Tensor) -> Tensor:
    """The fk image of W^T (the backward's dA = G W): the one the training forward packed beside W's
    if W is unchanged since, else packed now."""
    key = (W.data_ptr(), W._version, tuple(W.shape), W.device)
    hit = _PACKED.get(id(W))
    if hit is not None and hit[0]() is W and hit[1] == key and hit[3] is not None:
        return hit[3]
    return K.pack_weights(W.detach().t().contiguous(), fk_only=True)


def block_forward(
    Xv: Tensor,
    Xe: Tensor,
    src: Tensor,
    rev: Tensor,
    lay: DeviceLayout,
    weights: Sequence[Tensor],
    biases: Sequence[Optional[Tensor]],
    act: tuple[int, float],
    reduce: str,
    residual: bool,
    keep_states: bool = False,
    drop: Optional[tuple[float, int]] = None,
) -> tuple[Tensor, Tensor, list[tuple[Tensor, Tensor]]]:
    """Run the kernel sequence; returns (node, H_d, states) with states = [(H_l, S_l, amax_l)] for
    l = 0..d-1 (each layer's input hidden state, its aggregation and the fp32 split bounds (max|H_l|,
    max|S_l|) on the device, or an empty tensor) if keep_states, else [].
    drop = (p, seed): training-mode dropout of every layer update (layer l draws from
    dropout_offset(l, E, h))."""
    V = Xv.shape[0]
    amax = _amax_buffer(len(weights), Xv, reuse=not keep_states)
    a0 = None if amax is None else amax[0]
    if len(weights) == 0:
        H, _ = K.dmpnn_init(Xv, Xe, src)
        return _layers_forward(H, None, V, src, rev, lay, weights, biases, act, reduce, residual, keep_states,
                               drop)
    chunks = dst_chunks(lay)
    pitch = row_pitch(Xv.shape[1], Xv.dtype, chunks is not None) if (not keep_states and drop is None) else None
    if chunks is not None and Xv.dtype == torch.float32 and Xv.shape[1] >= 128 and Xv.shape[1] % 4 == 0:
        # hubs: the wave-per-node init for every node of in-degree <= MAX_FUSED_IN_DEGREE, then the
        # chunked init (the initial gather inside pass 1 of the chunked reduce) over the hubs' chunks
        # alone, so no wave walks a hub's hundreds of in-edges and H0 is written once
        H, S = K.dmpnn_init(Xv, Xe, src, lay.dst_ptr, lay.dst_perm, act=act, reduce=reduce, amax=a0, pitch=pitch,
                            skip_degree=MAX_FUSED_IN_DEGREE)
        K.dmpnn_init_chunked(Xv, Xe, src, lay.dst_ptr, lay.dst_perm, chunks, act=act, reduce=reduce,
                             amax=a0, pitch=pitch, H0=H, S=S, chunk_ids=hub_chunk_ids(lay, chunks))
    elif chunks is not None and Xv.dtype == torch.float32:
        # the chunked init over every node (h < 128: no wave-per-node init)
        H, S = K.dmpnn_init_chunked(Xv, Xe, src, lay.dst_ptr, lay.dst_perm, chunks, act=act, reduce=reduce, amax=a0,
                                    pitch=pitch)
    elif chunks is not None:
        H, _ = K.dmpnn_init(Xv, Xe, src, amax=a0)
        S = _aggregate(H, lay.dst_ptr, lay.dst_perm, V, reduce, act, chunks, amax=None if a0 is None else a0[1:2])
    else:
        H, S = K.dmpnn_init(Xv, Xe, src, lay.dst_ptr, lay.dst_perm, act=act, reduce=reduce, amax=a0, pitch=pitch)
    return _layers_forward(H, S, V, src, rev, lay, weights, biases, act, reduce, residual, keep_states, drop,
                           amax)


def row_pitch(h: int, dtype: torch.dtype, hubs: bool = False) -> Optional[int]:
    """Row pitch of the intermediate H_l / S_l of an inference forward: fp32 rows of h % 8 != 0 floats
    padded to a 32-byte multiple (h = 300 -> 304), so that no row shares a 32-B sector with its
    neighbour: the dst-ordered row stores of the init and of the layer kernels then write whole
    sectors, and every 16-B gather piece of a row lies in one sector (measured with tools/r5_pitch.sh:
    the layer kernel at h = 304 runs 113.5 us against 121.1 at h = 300, the same MFMA work).  None:
    dense rows (h % 8 == 0 already, bf16, h < 128, or NT_ROW_PAD=0).  Hub graphs (hubs: a node of
    in-degree > MAX_FUSED_IN_DEGREE, dst_chunks) pad to whole 128-byte L2 lines instead (h = 300 ->
    320): polymer-16 2.44 -> 2.39 ms per step, layer 658 -> 638 us (tools/r5_align.sh), while 128-B
    rows lose at config 2 (389 -> 404 us per step) and at qm9-32k (2.99 -> 3.07 ms, tools/r5_align2.sh)."""
    align = _ROW_ALIGN or (32 if hubs else 8)
    if dtype != torch.float32 or h % 4 or h % align == 0 or h < 128 or not _ROW_PAD:
        return None
    return (h + align - 1) // align * align


_NO_AMAX = torch.empty(0)  # a state without a valid amax row (bf16, or a path that skips the chain)
_ROW_PAD = os.environ.get("NT_ROW_PAD", "1") != "0"  # A/B: 0 = dense intermediate rows
_ROW_ALIGN = int(os.environ.get("NT_ROW_ALIGN", "0"))  # A/B: pitch multiple in floats (0: by graph size)


# fp32 relu / sum layers on graphs of at most this many edges take 64-row tiles walked by two 4-wave
# workgroups per CU (overlapping one's epilogue with the other's K loop); larger graphs keep the
# 128-row walk.  Measured per launch (tools/r4_sweep.sh, tools/r4_nw4b.sh): 78k edges 115-117 vs
# 125 us; 155k 243 vs 244; 310k 465 vs 462; 456k (polymer-16) 720 vs 691; 621k 904 vs 895.
NW4_MAX_EDGES = int(os.environ.get("NT_NW4_MAX_EDGES", "131072"))  # A/B override

# per (device, stream, depth): a ring of _AMAX_RING amax buffers for forwards that keep no states,
# zeroed all at once every _AMAX_RING forwards instead of one fill kernel per forward
_AMAX_RING = 64
_amax_rings: dict = {}
_amax_lock = threading.Lock()


def _amax_buffer(d: int, X: Tensor, reuse: bool = False) -> Optional[Tensor]:
    """(d + 1) x 2 zeros: row l = (max|H_l|, max|S_l|), the fp32 layer kernel's split scales (the
    init raises row 0, layer l reads row l and raises row l + 1).  None for bf16.
    reuse (forwards whose states nothing keeps): the next buffer of this stream's ring; the whole ring
    is zeroed when it wraps, which stream order makes safe (the forward that used a buffer last has
    finished before the fill that re-zeroes it runs).  Not while a graph is being captured (a replay
    must re-zero its own buffer)."""
    if X.dtype != torch.float32 or d == 0:
        return None
    if not reuse or torch.cuda.is_current_stream_capturing():
        return torch.zeros(d + 1, 2, dtype=torch.float32, device=X.device)
    key = (X.device, torch.cuda.current_stream(X.device).cuda_stream, d)
    with _amax_lock:  # threads sharing a stream take distinct slots; the wrap-time zeroing is enqueued once
        ent = _amax_rings.get(key)
        if ent is None:
            ent = _amax_rings[key] = [torch.empty(_AMAX_RING, d + 1, 2, dtype=torch.float32, device=X.device), 0]
        buf, i = ent
        if i == 0:
            buf.zero_()
        ent[1] = (i + 1) % _AMAX_RING
    return buf[i]


def dropout_offset(l: int, E: int, h: int) -> int:
    """First hash counter of layer l's dropout mask: layers draw disjoint counter ranges."""
    return l * E * h


def draw_dropout_seed() -> int:
    """One 62-bit seed from torch's default CPU generator (so torch.manual_seed reproduces masks)."""
    return int(torch.randint(0, 2**62, (1,), dtype=torch.int64).item())


def block_forward_embedded(
    node_table: Tensor,
    node_types: Tensor,
    edge_table: Tensor,
    edge_types: Tensor,
    src: Tensor,
    rev: Tensor,
    lay: DeviceLayout,
    weights: Sequence[Tensor],
    biases: Sequence[Optional[Tensor]],
    act: tuple[int, float],
    reduce: str,
    residual: bool,
    validate: bool = True,
) -> tuple[Tensor, Tensor]:
    """block_forward with GraphEmbedding fused into the initial gather (nt_dmpnn_init_embed):
    Xv / Xe are never materialised.  Returns (node, H_d)."""
    V = node_types.shape[0]
    if len(weights) == 0:
        H, _ = K.dmpnn_init_embed(node_table, node_types, edge_table, edge_types, src, validate=validate)
        node, H, _ = _layers_forward(H, None, V, src, rev, lay, weights, biases, act, reduce, residual, False)
        return node, H
    amax = _amax_buffer(len(weights), node_table, reuse=True)
    k72 = node_types.dim() == 2 and node_types.shape[1] == 7 and edge_types.dim() == 2 and edge_types.shape[1] == 2
    pitch = row_pitch(node_table.shape[1], node_table.dtype) if k72 else None
    rec = None
    if k72 and node_table.dtype == torch.float32 and embed_wave_ok(node_table.shape[0], edge_table.shape[0],
                                                                   node_table.shape[1]):
        rec = embed_records(lay, node_types, node_table.shape[0], edge_types, edge_table.shape[0], src)
    H, S = K.dmpnn_init_embed(node_table, node_types, edge_table, edge_types, src, lay.dst_ptr,
                              lay.dst_perm, act=act, reduce=reduce, validate=validate,
                              amax=None if amax is None else amax[0], pitch=pitch, records=rec)
    node, H, _ = _layers_forward(H, S, V, src, rev, lay, weights, biases, act, reduce, residual, False,
                                 amax=amax)
    return node, H


def _layers_forward(H, S, V, src, rev, lay, weights, biases, act, reduce, residual, keep_states, drop=None,
                    amax=None):
    """The d layers + final node scatter, from H0 and layer 0's aggregation S.  With dropout the
    update runs without its residual and nt_dropout_residual adds it back (the fused and persistent
    kernels write H_out directly, so dropout takes the unfused update).  amax (fp32): the split
    scales, row 0 filled by the init (see _amax_buffer)."""
    d = len(weights)
    chunks = dst_chunks(lay)
    if d == 0:
        node = _aggregate(H, lay.dst_ptr, lay.dst_perm, V, reduce, _IDENTITY, chunks)
        return node, H, []
    # a training forward (states kept for the kernel backward) packs the dA images of W^T alongside
    Wps = pack_layer_weights(weights, with_t=keep_states and H.dtype == torch.float32)
    E, h = H.shape
    fp32 = H.dtype == torch.float32
    if fp32 and amax is None:
        amax = _amax_buffer(d, H)
        K.absmax(H, amax[0, 0:1])
        K.absmax(S, amax[0, 1:2])
    fusable = drop is None and _fused_enabled() and K.fused_supported(V, E, h, H.dtype)
    rows = 64
    if fusable:  # the layer kernel's tile capacity for every layer of this block
        rows = min(K.fused_tile_rows(h, H.dtype, act, reduce, act),
                   K.fused_tile_rows(h, H.dtype, act, reduce, _IDENTITY))
        if rows == 128 and fp32 and h <= 320 and E <= NW4_MAX_EDGES and os.environ.get("NT_FK_NW") != "8":
            rows = 64  # the two-workgroups-per-CU walk of 64-row tiles (update_pk.hip, fk_nw4)
    plan = fused_plan(lay, V, E, rows, H.dtype) if fusable else None
    if plan is not None:
        return _fused_forward(H, S, src, rev, lay, plan, rows, Wps, biases, act, reduce, residual, keep_states,
                              amax)
    if not H.is_contiguous():  # row-padded init output (row_pitch) on a graph the fused plan cannot take
        H, S = H.contiguous(), S.contiguous()
    states = []
    spare: Optional[Tensor] = None  # ping-pong buffer when states are not kept
    # graphs the fused plan cannot take (in-degree > 32): fp32 still runs the persistent layer kernel,
    # without its aggregation (a separate segment reduce)
    persistent = fusable and fp32
    timer = UPDATE_EVENTS
    for l in range(d):
        if keep_states:  # the amax row is valid where the persistent kernel keeps the chain
            states.append((H, S, amax[l] if amax is not None and ((persistent and drop is None) or l == 0)
                           else _NO_AMAX))
        if timer is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        b_l = None if biases[l] is None else biases[l].detach()
        if drop is not None:
            U = K.dmpnn_update(H, S, src, rev, Wps[l], b_l, residual=False, act=act, out=spare)
            Hn = K.dropout_residual(U, drop[0], drop[1], dropout_offset(l, E, h),
                                    base=H if residual else None, out=U)
        elif persistent:  # the persistent kernel without its fused aggregation (hub graphs)
            Hn, _ = K.dmpnn_update_fused(H, S, src, rev, Wps[l], b_l, residual=residual, act=act,
                                         amax_in=amax[l], amax_out=amax[l + 1], out=spare)
        else:
            Hn = K.dmpnn_update(H, S, src, rev, Wps[l], b_l, residual=residual, act=act, out=spare)
        if timer is not None:
            ev[1].record()
            timer.append(ev)
        if l == 0:
            _note_update("persistent" if persistent else "unfused", H.dtype, h)
        if l < d - 1:
            S = _aggregate(Hn, lay.dst_ptr, lay.dst_perm, V, reduce, act, chunks,
                           out=None if keep_states else S, amax=amax[l + 1, 1:2] if persistent else None)
        if not keep_states:
            spare = H  # H_l is dead once H_{l+1} exists: reuse its buffer for H_{l+2}
        H = Hn
    node = _aggregate(H, lay.dst_ptr, lay.dst_perm, V, reduce, _IDENTITY, chunks)
    return node, H, states


def row_table(lay: DeviceLayout, dsts: Tensor, src: Tensor, rev: Tensor, V: int) -> Tensor:
    """The fp32 layer kernel's row table of this graph (nt_dmpnn_row_table), cached on the layout
    (keyed on the src storage and the rev_index tensor, like backward_layout)."""
    key = (src.data_ptr(), src.numel(), rev.data_ptr(), rev.numel(), V)
    hit = getattr(lay, "row_table", None)
    if hit is None or hit[0] != key or hit[1] is not rev:
        rt = K.dmpnn_row_table(lay.dst_perm, dsts, src, rev, V)
        hit = (key, rev, rt)
        lay.row_table = hit
    return hit[2]


EMBED_TABLE_BYTES = 72 * 1024  # LDS the wave-per-node embedding init holds the two tables in (embed.hip kTabB)


def embed_wave_ok(nv: int, ne: int, h: int) -> bool:
    """The wave-per-node fused embedding init applies (fp32, 7 + 2 type columns checked by the caller):
    both tables plus a zero row each fit its LDS, fewer than 255 types of each kind."""
    return h % 4 == 0 and h <= 512 and nv < 255 and ne < 255 and (nv + ne + 2) * h * 4 <= EMBED_TABLE_BYTES


def embed_records(lay: DeviceLayout, node_types: Tensor, nv: int, edge_types: Tensor, ne: int, src: Tensor) -> Tensor:
    """The graph's type records for the wave-per-node embedding init (kernels.embed_edge_records),
    cached on the layout, keyed on the type tensors (identity and version) and src."""
    key = (node_types.data_ptr(), node_types._version, edge_types.data_ptr(), edge_types._version,
           src.data_ptr(), src.numel(), nv, ne)
    hit = getattr(lay, "embed_records", None)
    if hit is None or hit[0] != key:
        hit = (key, K.embed_edge_records(node_types, nv, edge_types, ne, src, lay.dst_perm))
        lay.embed_records = hit
    return hit[1]


def hub_run_table(lay: DeviceLayout, rt: Tensor, tile_ptr: Tensor, dsts: Tensor, run_rows: int) -> tuple:
    """The row table with hub sub-runs (kernels.hub_runs) for this plan's tiles, cached on the layout
    (keyed on the base table and the plan): (table, nslots, hubs, slot_ptr)."""
    key = (rt.data_ptr(), tile_ptr.data_ptr(), tile_ptr.numel(), run_rows)
    hit = getattr(lay, "hub_runs", None)
    if hit is None or hit[0] != key:
        hit = (key, K.hub_runs(rt, lay.dst_ptr, dsts, tile_ptr, HUB_DEGREE, run_rows))
        lay.hub_runs = hit
    return hit[1]


def _fused_forward(H, S, src, rev, lay, plan, rows, Wps, biases, act, reduce, residual, keep_states, amax):
    tile_ptr, ntiles, dsts, zero_fill = plan
    # zero fills only where a row is read or returned (zero_rows_needed): the last layer's node output;
    # an intermediate S only if some source node has no in-edge
    zf_out, zf_mid, _ = zero_rows_needed(lay, src, S.shape[0]) if zero_fill else (False, False, False)
    d = len(Wps)
    rt = row_table(lay, dsts, src, rev, S.shape[0])
    states = []
    spare_H: Optional[Tensor] = None
    spare_S: Optional[Tensor] = None
    timer = UPDATE_EVENTS
    maxdeg = fused_max_in_degree(lay)
    hubs = hub_info(lay)
    part = None
    if hubs is not None:  # hub sub-runs: the layer writes their partials, hub_combine finishes the hubs
        rt, nslots, hub_ids, slot_ptr = hub_run_table(lay, rt, tile_ptr, dsts, max(1, maxdeg))
        part = torch.empty(max(nslots, 1), H.shape[1], dtype=torch.float32, device=H.device)
    for l in range(d):
        last = l == d - 1
        if keep_states:
            states.append((H, S, _NO_AMAX if amax is None else amax[l]))
        if timer is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        # intermediate layers keep the input's row pitch (row_pitch); the block's outputs are dense
        pitch = H.shape[1] if last else H.stride(0)
        if spare_H is not None and spare_H.stride(0) != pitch:
            spare_H = spare_S = None
        Hn, Sn = K.dmpnn_update_fused(
            H, S, src, rev, Wps[l], None if biases[l] is None else biases[l].detach(),
            residual=residual, act=act, plan=(tile_ptr, ntiles, dsts), tile_rows=rows, max_in_degree=maxdeg,
            perm=lay.dst_perm, reduce=reduce, agg_act=_IDENTITY if last else act,
            zero_fill=zf_out if last else zf_mid,
            amax_in=None if amax is None else amax[l],
            amax_out=None if (amax is None or last) else amax[l + 1],  # row d has no reader
            row_table=rt, out=spare_H, S_out=None if last else spare_S, pitch_out=pitch, S_part=part,
        )
        if timer is not None:
            ev[1].record()
            timer.append(ev)
        if hubs is not None:  # the hubs' S_out rows from the launch's sub-run partials
            K.hub_combine(part, hub_ids, slot_ptr, lay.dst_ptr, Sn, reduce=reduce,
                          amax=None if (amax is None or last) else amax[l + 1, 1:2])
        if l == 0:
            _note_update("fused", H.dtype, H.shape[1], rows)
        if not keep_states:
            spare_H = H
            spare_S = S
        H, S = Hn, Sn
    return S, H, states


# ------------------------------------------------------------------------------------ autograd
def _torch_scatter(x: Tensor, index: Tensor, dim_size: int, reduce: str) -> Tensor:
    """torch_scatter.scatter semantics (empty segment -> 0) in device ops, for the backward."""
    out = torch.zeros(dim_size, x.shape[1], dtype=x.dtype, device=x.device)
    idx = index.view(-1, 1).expand_as(x)
    if reduce == "sum":
        return out.scatter_add(0, idx, x)
    red = {"mean": "mean", "max": "amax", "min": "amin"}[reduce]
    return out.scatter_reduce(0, idx, x, reduce=red, include_self=False)


def _torch_block(Xv, Xe, edge_index, rev, weights, biases, act_mod, reduce, residual, masks=None):
    src, dst = edge_index[0], edge_index[1]
    V = Xv.shape[0]
    H = Xv[src] + Xe
    for l, (W, b) in enumerate(zip(weights, biases)):
        M = act_mod(H)
        S = _torch_scatter(M, dst, V, reduce)
        U = torch.nn.functional.linear(S[src] - M[rev], W, b)
        if masks is not None:  # dropout: keep / (1 - p), regenerated by the kernel's hash
            U = U * masks[l]
        H = H + U if residual else U
    return _torch_scatter(H, dst, V, reduce), H


# ------------------------------------------------------------------------------------ layerwise
# Blocks the fused kernels do not take as one unit: an activation outside the kernels' codes (any
# nn.Module, chemprop.py:17,24,37), or layers that differ in activation or dropout.  Every layer
# runs unfused on the device: M = act(H) as the module's own elementwise op when it has no kernel
# code, then the segment-reduce and update kernels on M with the identity activation
# (S = scatter(M, dst), U = W (S[src] - M[rev]) + b), dropout by the hash kernel, residual add.
def layer_act(act_mod: torch.nn.Module) -> Optional[tuple[int, float]]:
    try:
        return K.act_code(act_mod)
    except NotImplementedError:
        return None


def block_forward_layerwise(Xv, Xe, src, rev, lay, acts, weights, biases, drops, reduce, residual):
    """acts[l] = (module, kernel code or None); drops[l] = (p, seed) or None.  Returns (node, H_d)."""
    V = Xv.shape[0]
    H, _ = K.dmpnn_init(Xv, Xe, src)
    chunks = dst_chunks(lay)
    E, h = H.shape
    for l, ((mod, code), W, b) in enumerate(zip(acts, weights, biases)):
        if code is None:
            M, code_l = mod(H).contiguous(), _IDENTITY
        else:
            M, code_l = H, code
        S = _aggregate(M, lay.dst_ptr, lay.dst_perm, V, reduce, code_l, chunks)
        Wp = pack_layer_weights([W])[0]
        U = K.dmpnn_update(M, S, src, rev, Wp, None if b is None else b.detach(), residual=False, act=code_l)
        if drops[l] is not None:
            H = K.dropout_residual(U, drops[l][0], drops[l][1], dropout_offset(l, E, h),
                                   base=H if residual else None, out=U)
        else:
            H = H + U if residual else U
    node = _aggregate(H, lay.dst_ptr, lay.dst_perm, V, reduce, _IDENTITY, chunks)
    return node, H


def _torch_block_layerwise(Xv, Xe, edge_index, rev, weights, biases, act_mods, reduce, residual, masks):
    src, dst = edge_index[0], edge_index[1]
    V = Xv.shape[0]
    H = Xv[src] + Xe
    for l, (W, b) in enumerate(zip(weights, biases)):
        M = act_mods[l](H)
        S = _torch_scatter(M, dst, V, reduce)
        U = torch.nn.functional.linear(S[src] - M[rev], W, b)
        if masks[l] is not None:
            U = U * masks[l]
        H = H + U if residual else U
    return _torch_scatter(H, dst, V, reduce), H


class LayerwiseBlockFunction(torch.autograd.Function):
    """Kernel forward (block_forward_layerwise); backward by recomputing the same math in PyTorch
    device ops under autograd (any activation module, per-layer dropout masks regenerated by the
    hash kernel).  The activation modules' own parameters (e.g. nn.PReLU's slope) are inputs of
    the Function and get their gradients from the recompute; the RNG state of the forward is
    restored for the recompute, so a stochastic activation (nn.RReLU in training) draws the same
    values in both."""

    @staticmethod
    def forward(ctx, Xv, Xe, edge_index, rev, lay, acts, drops, reduce, residual, nlayers, nact, *params):
        weights, biases = list(params[:nlayers]), list(params[nlayers:2 * nlayers])
        dev = Xv.device
        ctx.rng = (torch.get_rng_state(), torch.cuda.get_rng_state(dev))
        node, H = block_forward_layerwise(Xv, Xe, edge_index[0].contiguous(), rev, lay, acts, weights,
                                          biases, drops, reduce, residual)
        ctx.save_for_backward(Xv, Xe, edge_index, rev, *[p if p is not None else torch.empty(0) for p in params])
        ctx.cfg = (acts, drops, reduce, residual, nlayers, nact, [p is None for p in params])
        return node, H

    @staticmethod
    def backward(ctx, dnode, dH):
        acts, drops, reduce, residual, nlayers, nact, is_none = ctx.cfg
        Xv, Xe, edge_index, rev, *rest = ctx.saved_tensors
        params = [None if n else p for p, n in zip(rest, is_none)]
        need = ctx.needs_input_grad
        nfix = 11  # inputs of forward() before *params
        dev = Xv.device
        with torch.enable_grad(), torch.random.fork_rng(devices=[dev]):
            torch.set_rng_state(ctx.rng[0])
            torch.cuda.set_rng_state(ctx.rng[1], dev)
            Xv_ = Xv.detach().requires_grad_(need[0])
            Xe_ = Xe.detach().requires_grad_(need[1])
            ps = [None if p is None else p.detach().requires_grad_(True) for p in params[:2 * nlayers]]
            # activation parameters: the module's own tensors (the recompute calls the modules)
            aps = params[2 * nlayers:]
            E, h = Xe.shape
            masks = [None if d is None else K.dropout_residual(torch.ones_like(Xe), d[0], d[1], dropout_offset(l, E, h))
                     for l, d in enumerate(drops)]
            node, H = _torch_block_layerwise(Xv_, Xe_, edge_index, rev, ps[:nlayers], ps[nlayers:],
                                             [a[0] for a in acts], reduce, residual, masks)
            act_leaves = [p for i, p in enumerate(aps) if p is not None and need[nfix + 2 * nlayers + i]]
            leaves = [t for t in [Xv_, Xe_] + ps if t is not None and t.requires_grad] + act_leaves
            outs, grads = [], []
            for o, g in ((node, dnode), (H, dH)):
                if g is not None:
                    outs.append(o)
                    grads.append(g)
            got = torch.autograd.grad(outs, leaves, grads, allow_unused=True)
        it = iter(got)
        res_inputs = [next(it) if need[0] else None, next(it) if need[1] else None]
        res_params = [None if p is None else next(it) for p in ps]
        res_params += [next(it) if p is not None and need[nfix + 2 * nlayers + i] else None
                       for i, p in enumerate(aps)]
        return (*res_inputs, None, None, None, None, None, None, None, None, None, *res_params)


def dA_plan(lay: DeviceLayout, src: Tensor, V: int, E: int, src_ptr: Tensor, src_perm: Tensor):
    """The backward's fused dA + dS launch plan (fp32): node-aligned 64-row tiles over the src-sorted
    edge order (the transpose of the forward's dst plan) and its row table {edge, e, -1, src node}:
    A[e] = G[e] (the "src" row of the gather is the edge itself, nothing subtracted), so the layer
    kernel's fused mode computes dA = G W and dS[v] = sum_{e: src[e] = v} dA[e] in ascending edge order
    (the bits of segment_reduce(dA, src CSR)).  None when some node has more than
    MAX_FUSED_IN_DEGREE out-edges (then dense_matmul + segment_reduce).  Cached on the layout."""
    key = (src.data_ptr(), src.numel(), V)
    hit = getattr(lay, "da_plan", None)
    if hit is None or hit[0] != key:
        plan = None
        if E > 0 and V > 0:
            outdeg = src_ptr[1:] - src_ptr[:-1]
            dmax, dmin = int(outdeg.max()), int(outdeg.min())
            if dmax <= MAX_FUSED_IN_DEGREE:
                tile_ptr, ntiles, dsts = K.tile_plan(src_ptr, E, dmax, rows=64, ncu=K.PLAN_SLOTS64)
                ident = torch.arange(E, dtype=torch.int64, device=src.device)
                none = torch.full((E,), -1, dtype=torch.int64, device=src.device)
                # the gathered operand is G (E rows): the row table's bound on the "src" index is E
                rt = K.dmpnn_row_table(src_perm, dsts, ident, none, E)
                # dS rows no tile writes (out-degree 0) need zeros only if an edge's dS[dst] reads them
                zf = dmin == 0 and zero_rows_needed(lay, src, V)[2]
                plan = ((tile_ptr, ntiles, dsts), dmax, zf, ident, none, rt)
        hit = (key, plan)
        lay.da_plan = hit
    return hit[1]


def backward_layout(lay: DeviceLayout, src: Tensor, rev: Tensor, V: int, E: int) -> tuple:
    """(src_ptr, src_perm, rev_ptr, rev_perm): the CSRs of the two gathers' transposes (scatter by
    src into nodes, scatter by rev_index into edges), built once per graph and cached on its layout."""
    bwd = getattr(lay, "bwd", None)
    # keyed on the storage (src is a fresh view of edge_index[0] on every call) and the rev tensor
    key = (src.data_ptr(), src.numel(), rev.data_ptr(), rev.numel(), V)
    if bwd is None or bwd[0] != key or bwd[1] is not rev:
        src_ptr, src_perm = K.csr_build(src, V, check_bounds=False)
        rev_ptr, rev_perm = K.csr_build(rev, E, check_bounds=False)
        bwd = (key, rev, src_ptr, src_perm, rev_ptr, rev_perm)
        lay.bwd = bwd
    return bwd[2:]


def _weight_grad(G: Tensor, A: Tensor) -> Tensor:
    """dW = G^T A (h x h, reduction over all E edges).  A single GEMM has only (h/32)(h/64) output
    tiles, far too few for 256 CUs, so the edge dimension is split k ways into a batched GEMM
    whose k partial products are then summed (split-K)."""
    E, h = G.shape
    k = min(64, E // 2048)
    if k < 2:
        return torch.mm(G.t(), A)
    rows = E // k
    Eb = rows * k
    # bf16: the k partials are summed in fp32 and rounded once
    dW = torch.bmm(G[:Eb].view(k, rows, h).transpose(1, 2), A[:Eb].view(k, rows, h)).sum(
        0, dtype=torch.float32).to(G.dtype)
    if Eb < E:
        dW.addmm_(G[Eb:].t(), A[Eb:])
    return dW


def block_backward(dnode, dH, states, weights, src, dst, rev, lay, act, reduce, residual, V, need_x,
                   drop=None, H_last=None):
    """Kernel backward of block_forward (see csrc/backward.hip), fp32 or bf16 storage, every reduce:
    max / min aggregations send each gradient element to its arg (torch_scatter's scatter_max /
    scatter_min): H_last = the forward's H_d, for the final node scatter's arg.
    Returns (dXv, dXe, [dW_l], [db_l])."""
    maxmin = reduce in ("max", "min")
    E, h = states[0][0].shape if states else (dH.shape if dH is not None else (rev.numel(), dnode.shape[1]))
    src_ptr, src_perm, rev_ptr, rev_perm = backward_layout(lay, src, rev, V, E)
    mean_ptr = lay.dst_ptr if reduce == "mean" else None
    d = len(weights)
    gdtype = dH.dtype if dH is not None else (dnode.dtype if dnode is not None else states[0][0].dtype)
    # G = dL/dH_d: the gather of dnode below writes it whole when H_d itself has no gradient (no
    # E x h zero fill to add it to)
    G = dH.contiguous() if dH is not None else None
    if G is None and dnode is None:
        G = torch.zeros(E, h, dtype=gdtype, device=src.device)
    # fp32: max|G| of the current G, raised by the kernel that writes G (the fp16-split kernels'
    # scale); None = unknown (nt_absmax computes it).  One zero-filled buffer for every layer's row.
    fp32 = gdtype == torch.float32
    gbuf = torch.zeros(d + 1, 2, dtype=torch.float32, device=src.device) if fp32 else None
    gmax_cur = None
    if dnode is not None:
        gmax_cur = None if gbuf is None else gbuf[d]
        g1 = None if gmax_cur is None else gmax_cur[1:2]
        if maxmin:  # chemprop.py:86 with scatter_max / scatter_min
            arg = K.segment_arg(H_last, lay.dst_ptr, lay.dst_perm, V, reduce)
            G = K.gather_rows_arg(dnode.contiguous(), dst, arg, base=G, amax=g1)
        else:
            G = K.gather_rows(dnode.contiguous(), dst, base=G, seg_ptr=mean_ptr, amax=g1)
    dWs: list = [None] * d
    dbs: list = [None] * d
    wgrad = os.environ.get("NT_WGRAD", _WGRAD_DEFAULT)
    for l in range(d - 1, -1, -1):
        H_l, S_l, am_l = states[l]
        W = weights[l].detach()
        # dropout: the update's gradient is keep * G / (1 - p); the residual path keeps G
        Gu = G if drop is None else K.dropout_residual(G, drop[0], drop[1], dropout_offset(l, E, h))
        Gu = Gu.contiguous()
        fk_dense = fp32 and K.fused_supported(V, E, h, Gu.dtype)
        fk_wgrad = fp32 and wgrad == "kernel" and h <= 320
        bf16_kernels = Gu.dtype == torch.bfloat16 and wgrad != "library" and h <= 512 and h % 8 == 0
        gmax = gmax_cur if drop is None else None  # dropout rescales G: its max is taken afresh
        if (fk_dense or fk_wgrad) and gmax is None:  # max|G|: the split scale of both fp16-split kernels
            gmax = torch.zeros(2, dtype=torch.float32, device=Gu.device)
            K.absmax(Gu, gmax[1:2])
        if fp32 and wgrad in ("kernel", "kernel6"):
            # split-K MFMA with A = S[src] - act(H[rev]) formed while staging (never written): the
            # two-part fp16 kernel (h <= 320) on the forward's bounds, else bf16x6
            am = None
            if fk_wgrad:
                am = am_l if am_l.numel() == 2 else None
                if am is None:  # a forward path that did not keep the chain
                    am = torch.zeros(2, dtype=torch.float32, device=Gu.device)
                    K.absmax(H_l.contiguous(), am[0:1])
                    K.absmax(S_l.contiguous(), am[1:2])
            dWs[l], dbs[l] = K.weight_grad(Gu, H_l.contiguous(), S_l.contiguous(), src, rev, act=act,
                                           amax_G=None if am is None else gmax[1:2], amax_HS=am)
        elif bf16_kernels:  # A rounded to bf16 in the kernel as the forward's message; fp32 partials
            dW32, db32 = K.weight_grad(Gu, H_l.contiguous(), S_l.contiguous(), src, rev, act=act)
            dWs[l], dbs[l] = dW32.to(Gu.dtype), db32.to(Gu.dtype)
        else:
            A = K.dmpnn_message(H_l, S_l, src, rev, act=act)
            dWs[l] = _weight_grad(Gu, A)
            dbs[l] = Gu.sum(0)
            del A
        dap = dA_plan(lay, src, V, E, src_ptr, src_perm) if (fk_dense and _FUSED_DA) else None
        if dap is not None:
            # dA = G W and dS = sum_src dA in one launch of the layer kernel's fused mode over the
            # src-sorted plan (A[e] = G[e]: rev = -1 everywhere, so act and H are never applied)
            plan3, dmax, zf, ident, none, rt = dap
            # gmax = (0, max|G|): [0] is never written (the bound of the H term, absent here), so the
            # split scale is dense_matmul's
            amx = gmax
            dS = (torch.zeros if zf else torch.empty)(V, h, dtype=Gu.dtype, device=Gu.device)
            dA, dS = K.dmpnn_update_fused(Gu, Gu, ident, none, packed_transpose(weights[l]), None,
                                          residual=False, act=_RELU, plan=plan3, tile_rows=64, max_in_degree=dmax,
                                          perm=src_perm, reduce="sum", agg_act=_IDENTITY, amax_in=amx,
                                          row_table=rt, S_out=dS, n_nodes=V)
        else:
            if fk_dense:
                dA = K.dense_matmul(Gu, packed_transpose(weights[l]), amax=gmax)
            elif bf16_kernels and os.environ.get("NT_BF16_DA", "kernel") == "kernel":  # the bf16 layer kernel
                dA = K.dense_matmul(Gu, K.pack_weights(W.t().contiguous()))  # without gathers
            else:
                dA = torch.mm(Gu, W)
            dS = K.segment_reduce(dA, src_ptr, src_perm, V, reduce="sum", act=_IDENTITY)
        del Gu
        gmax_cur = gbuf[l - 1] if fp32 and l > 0 else None
        g1 = None if gmax_cur is None else gmax_cur[1:2]
        if maxmin:  # chemprop.py:39 with scatter_max / scatter_min: the arg of act(H_l) per node
            arg = K.segment_arg(H_l, lay.dst_ptr, lay.dst_perm, V, reduce, act=act)
            G = K.dmpnn_edge_backward_arg(G, H_l, dA, dS, arg, dst, rev_ptr, rev_perm,
                                          residual=residual, act=act, amax=g1)
        else:
            G = K.dmpnn_edge_backward(G, H_l, dA, dS, dst, rev_ptr, rev_perm, lay.dst_ptr,
                                      residual=residual, act=act, reduce=reduce, amax=g1)
    dXv = K.segment_reduce(G, src_ptr, src_perm, V, reduce="sum", act=_IDENTITY) if need_x[0] else None
    return dXv, G if need_x[1] else None, dWs, dbs


class ChempropBlockFunction(torch.autograd.Function):
    """Kernel forward; kernel backward (block_backward: gather / scatter / element-wise HIP kernels and
    the MFMA dA / dW kernels) for every reduce in fp32 and bf16 storage; NT_BWD=torch selects the
    recompute-in-torch-device-ops backward (an A/B reference only)."""

    @staticmethod
    def forward(ctx, Xv, Xe, edge_index, rev, lay, act_mod, act, reduce, residual, nlayers, drop, *params):
        weights = list(params[:nlayers])
        biases = list(params[nlayers:])
        src = edge_index[0].contiguous()
        kernel_bwd = (reduce in ("sum", "mean", "max", "min") and Xv.dtype in (torch.float32, torch.bfloat16)
                      and os.environ.get("NT_BWD", "kernel") != "torch")
        node, H, states = block_forward(Xv, Xe, src, rev, lay, weights, biases, act, reduce, residual,
                                        keep_states=kernel_bwd, drop=drop)
        flat = [t for hs in states for t in hs]
        if kernel_bwd and reduce in ("max", "min"):
            flat.append(H)  # the final node scatter's arg is taken over H_d
        ctx.save_for_backward(Xv, Xe, edge_index, rev,
                              *[p if p is not None else torch.empty(0) for p in params], *flat)
        ctx.cfg = (act_mod, act, reduce, residual, nlayers, [p is None for p in params], lay, kernel_bwd, drop)
        # an output the loss does not use arrives as None instead of an E x h zero tensor: the backward
        # then writes G = dnode[dst] whole (no zero fill, no zero base read by the gather)
        ctx.set_materialize_grads(False)
        return node, H

    @staticmethod
    def backward(ctx, dnode, dH):
        act_mod, act, reduce, residual, nlayers, is_none, lay, kernel_bwd, drop = ctx.cfg
        Xv, Xe, edge_index, rev, *rest = ctx.saved_tensors
        nparams = len(is_none)
        params = [None if n else p for p, n in zip(rest[:nparams], is_none)]
        need = ctx.needs_input_grad
        if dnode is None and dH is None:  # set_materialize_grads(False): neither output reached the loss
            return (None,) * (11 + nparams)
        if kernel_bwd:
            flat = rest[nparams:]
            states = [tuple(flat[3 * i:3 * i + 3]) for i in range(nlayers)]
            H_last = flat[3 * nlayers] if reduce in ("max", "min") else None
            src = edge_index[0].contiguous()
            dst = edge_index[1].contiguous()
            dXv, dXe, dWs, dbs = block_backward(
                dnode, dH, states, params[:nlayers], src, dst, rev, lay, act, reduce, residual,
                Xv.shape[0], (need[0], need[1]), drop, H_last,
            )
            res_params = [dW if need[11 + i] else None for i, dW in enumerate(dWs)]
            res_params += [None if p is None or not need[11 + nlayers + i] else dbs[i]
                           for i, p in enumerate(params[nlayers:])]
            return (dXv, dXe, None, None, None, None, None, None, None, None, None, *res_params)
        with torch.enable_grad():
            Xv_ = Xv.detach().requires_grad_(need[0])
            Xe_ = Xe.detach().requires_grad_(need[1])
            ps = [None if p is None else p.detach().requires_grad_(True) for p in params]
            masks = None
            if drop is not None:
                E, h = Xe.shape
                ones = torch.ones_like(Xe)
                masks = [K.dropout_residual(ones, drop[0], drop[1], dropout_offset(l, E, h))
                         for l in range(nlayers)]
            node, H = _torch_block(Xv_, Xe_, edge_index, rev, ps[:nlayers], ps[nlayers:], act_mod, reduce,
                                   residual, masks)
            leaves = [t for t in [Xv_, Xe_] + ps if t is not None and t.requires_grad]
            outs, grads = [], []
            for o, g in ((node, dnode), (H, dH)):
                if g is not None:
                    outs.append(o)
                    grads.append(g)
            got = torch.autograd.grad(outs, leaves, grads, allow_unused=True)
        it = iter(got)
        res_inputs = [next(it) if need[0] else None, next(it) if need[1] else None]
        res_params = [None if p is None else next(it) for p in ps]
        return (*res_inputs, None, None, None, None, None, None, None, None, None, *res_params)


def mol_chunks(G, mol_ptr: Tensor):
    """Chunk plan of the molecule CSR when some molecule has more than LONG_SEGMENT atoms (polymers,
    config 5), else None; cached on the layout with the molecule CSR it belongs to."""
    lay = getattr(G, "_nt_layout", None)
    hit = getattr(lay, "mol_chunks", None) if lay is not None else None
    if hit is not None and hit[0] is mol_ptr:
        return hit[1] or None
    n = mol_ptr[1:] - mol_ptr[:-1]
    ch = False
    if n.numel() and int(n.max()) > LONG_SEGMENT:
        ch = K.chunk_plan(mol_ptr)
    if lay is not None:
        lay.mol_chunks = (mol_ptr, ch)
    return ch or None


def segment_reduce_readout(X: Tensor, mol_ptr: Tensor, mol_perm: Optional[Tensor], B: int, reduce: str,
                           batch_node_index: Tensor, chunks=None) -> Tensor:
    if torch.is_grad_enabled() and X.requires_grad:
        return ReadoutFunction.apply(X, mol_ptr, mol_perm, B, reduce, batch_node_index, chunks)
    return _aggregate(X, mol_ptr, mol_perm, B, reduce, _IDENTITY, chunks)


class ReadoutFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, mol_ptr, mol_perm, B, reduce, batch_node_index, chunks=None):
        ctx.save_for_backward(X, batch_node_index)
        ctx.cfg = (B, reduce, mol_ptr)
        ctx.mol_perm = mol_perm
        return _aggregate(X, mol_ptr, mol_perm, B, reduce, _IDENTITY, chunks)

    @staticmethod
    def backward(ctx, dout):
        X, bni = ctx.saved_tensors
        B, reduce, mol_ptr = ctx.cfg
        if reduce in ("sum", "mean") and dout.dtype in (torch.float32, torch.bfloat16):
            # dX[v] = dout[batch v] (/ count for mean): one gather kernel
            dX = K.gather_rows(dout.contiguous(), bni, seg_ptr=mol_ptr if reduce == "mean" else None)
            return dX, None, None, None, None, None, None
        if reduce in ("max", "min") and dout.dtype in (torch.float32, torch.bfloat16):
            # agg.py:45 scatter_max: dX[v] = dout[batch v] where v is the molecule's arg
            mol_perm = ctx.mol_perm
            arg = K.segment_arg(X.contiguous(), mol_ptr, mol_perm, B, reduce)
            dX = K.gather_rows_arg(dout.contiguous(), bni, arg)
            return dX, None, None, None, None, None, None
        with torch.enable_grad():
            X_ = X.detach().requires_grad_(True)
            out = _torch_scatter(X_, bni, B, reduce)
            (dX,) = torch.autograd.grad(out, X_, dout)
        return dX, None, None, None, None, None, None
