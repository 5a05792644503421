"""Tensor-level wrappers over the C-ABI (``include/notorch_amd.h``).

Each wrapper validates device / dtype / shape / contiguity up front (raising ``TypeError`` /
``ValueError`` the way the reference's ATen ops would raise for bad inputs), allocates outputs with
``torch.empty`` on the tensor's device (PyTorch's caching allocator owns all memory) and launches on
``torch.cuda.current_stream()``.  Nothing here computes on the host: a CPU tensor is an error.
"""
from __future__ import annotations

import ctypes

import torch
from torch import Tensor

from notorch_amd import _lib
from notorch_amd._lib import NT_BF16, NT_F32, REDUCE_CODES, check

__all__ = [
    "csr_build",
    "dmpnn_init",
    "segment_reduce",
    "dmpnn_aggregate",
    "chunk_plan",
    "pack_weights",
    "dmpnn_update",
    "tile_plan",
    "tile_stride",
    "fused_tile_rows",
    "absmax",
    "dmpnn_row_table",
    "fused_supported",
    "dmpnn_update_fused",
    "act_code",
    "reduce_code",
    "dmpnn_message",
    "dmpnn_edge_backward",
    "gather_rows",
    "embed_bag",
    "dmpnn_init_embed",
    "embed_edge_records",
    "node_scores",
    "softmax_pool",
    "dense_matmul",
    "weight_grad",
    "segment_arg",
    "dmpnn_edge_backward_arg",
    "gather_rows_arg",
]


def _ptr(t: Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _run(dev: torch.device, fn, *args) -> None:
    """Call a C-ABI entry point with ``dev`` as the current HIP device (the library queries the
    current device for its CU count and kernel attributes; the launch goes to dev's stream)."""
    if dev.index is not None and dev.index != torch.cuda.current_device():
        with torch.cuda.device(dev):
            check(fn(*args))
    else:
        check(fn(*args))


def _require_device(*ts: Tensor | None) -> torch.device:
    dev = None
    for t in ts:
        if t is None:
            continue
        if t.device.type != "cuda":
            raise RuntimeError(
                "notorch_amd kernels run on ROCm devices only; got a tensor on "
                f"'{t.device}'. Move the graph with G.to('cuda') first."
            )
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise ValueError(f"tensors on different devices: {dev} vs {t.device}")
    assert dev is not None
    return dev


def _require_f32(name: str, t: Tensor) -> None:
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32 on the fp32 kernel path, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


_DTYPE_CODES = {torch.float32: NT_F32, torch.bfloat16: NT_BF16}


def _require_feat(name: str, t: Tensor, dtype: torch.dtype | None = None) -> int:
    """Feature tensor on the kernel path: fp32 or bf16 (all operands of one call share it), contiguous.
    Returns the C-ABI dtype code."""
    if t.dtype not in _DTYPE_CODES:
        raise TypeError(f"{name} must be float32 or bfloat16, got {t.dtype}")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name} is {t.dtype} but the other operands are {dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return _DTYPE_CODES[t.dtype]


def _row_pitch(name: str, t: Tensor, dtype: torch.dtype | None = None) -> int:
    """Row pitch (elements) of a 2-D feature tensor that is contiguous or a row-padded view
    (X[:, :h] of an [n, ld] fp32 buffer: unit column stride, 16-byte row pitch)."""
    if t.dim() != 2:
        raise ValueError(f"{name} must be 2-D")
    if t.is_contiguous():
        _require_feat(name, t, dtype)
        return t.shape[1]
    if t.dtype != torch.float32 or t.stride(1) != 1 or t.stride(0) < t.shape[1] or t.stride(0) % 4:
        raise ValueError(f"{name} must be contiguous (or an fp32 row-padded view with a pitch % 4 == 0)")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name} is {t.dtype} but the other operands are {dtype}")
    return t.stride(0)


def padded_rows(n: int, h: int, pitch: int, dtype: torch.dtype, device) -> Tensor:
    """An n x h tensor whose rows sit ``pitch`` elements apart (a view of an n x pitch buffer)."""
    if pitch == h:
        return torch.empty(n, h, dtype=dtype, device=device)
    return torch.empty(max(n, 1), pitch, dtype=dtype, device=device)[:n, :h]


def _require_i64(name: str, t: Tensor) -> None:
    if t.dtype != torch.int64:
        raise TypeError(f"{name} must be int64 (reference index dtype), got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def reduce_code(reduce: str) -> int:
    try:
        return REDUCE_CODES[reduce]
    except KeyError:
        raise ValueError(f"unsupported reduce '{reduce}', expected one of {list(REDUCE_CODES)}")


def act_code(act: torch.nn.Module) -> tuple[int, float]:
    """Map an activation module instance to the kernel's (code, alpha)."""
    nn = torch.nn
    if isinstance(act, nn.ReLU):
        return _lib.NT_ACT_RELU, 0.0
    if isinstance(act, nn.Identity):
        return _lib.NT_ACT_IDENTITY, 0.0
    if isinstance(act, nn.LeakyReLU):
        return _lib.NT_ACT_LEAKY_RELU, float(act.negative_slope)
    if isinstance(act, nn.ELU):
        return _lib.NT_ACT_ELU, float(act.alpha)
    if isinstance(act, nn.GELU):
        if act.approximate != "none":
            raise NotImplementedError("GELU(approximate='tanh') is not implemented in the kernels")
        return _lib.NT_ACT_GELU, 0.0
    if isinstance(act, nn.SiLU):
        return _lib.NT_ACT_SILU, 0.0
    if isinstance(act, nn.Tanh):
        return _lib.NT_ACT_TANH, 0.0
    if isinstance(act, nn.Sigmoid):
        return _lib.NT_ACT_SIGMOID, 0.0
    raise NotImplementedError(
        f"activation {type(act).__name__} has no kernel implementation "
        "(supported: ReLU, Identity, LeakyReLU, ELU, GELU, SiLU, Tanh, Sigmoid)"
    )


def csr_build(idx: Tensor, nseg: int, *, check_bounds: bool = True) -> tuple[Tensor, Tensor]:
    """Stable CSR of an int64 index vector: (seg_ptr[nseg+1] int32, perm[n] int32).

    ``check_bounds`` synchronises once to raise ``IndexError`` for out-of-range indices, like the
    reference's scatter would; the kernel itself never reads or writes out of bounds.
    """
    dev = _require_device(idx)
    _require_i64("idx", idx)
    if idx.dim() != 1:
        raise ValueError("idx must be 1-D")
    n = idx.numel()
    if nseg < 0:
        raise ValueError("nseg must be >= 0")
    lib = _lib.load()
    seg_ptr = torch.empty(nseg + 1, dtype=torch.int32, device=dev)
    perm = torch.empty(max(n, 1), dtype=torch.int32, device=dev)[:n]
    ws_bytes = lib.nt_csr_workspace_bytes(n, nseg)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    _run(dev, lib.nt_csr_build,
         _ptr(idx), n, nseg, _ptr(seg_ptr), _ptr(perm), _ptr(ws), ws_bytes, _ptr(err), _stream(dev))
    if check_bounds and n > 0 and int(err.item()) != 0:
        raise IndexError(f"index out of range for a scatter into {nseg} rows")
    return seg_ptr, perm


def dmpnn_init(
    Xv: Tensor,
    Xe: Tensor,
    src: Tensor,
    seg_ptr: Tensor | None = None,
    perm: Tensor | None = None,
    *,
    act: tuple[int, float] = (_lib.NT_ACT_RELU, 0.0),
    reduce: str = "sum",
    amax: Tensor | None = None,
    pitch: int | None = None,
    skip_degree: int = 0,
) -> tuple[Tensor, Tensor | None]:
    """H0 = Xv[src] + Xe, optionally fused with S = scatter(act(H0), dst) (needs the dst CSR).
    skip_degree (fp32, with S, h >= 128): nodes with more in-edges are left out (their H0 rows and S
    row are then dmpnn_init_chunked's with chunk_ids = their chunks).
    amax (fp32, 2 zero-filled device floats): raised to max|H0|, max|S| (layer 0's amax_in).
    pitch (fp32, h % 4 == 0, h >= 128 with the aggregation): H0 and S as row-padded views whose rows
    sit ``pitch`` floats apart (nt_dmpnn_init's ld_out)."""
    dev = _require_device(Xv, Xe, src, seg_ptr, perm, amax)
    _require_amax(amax, Xv.dtype)
    code = _require_feat("node_feats", Xv)
    _require_feat("edge_feats", Xe, Xv.dtype)
    _require_i64("src", src)
    if Xv.dim() != 2 or Xe.dim() != 2 or Xv.shape[1] != Xe.shape[1]:
        raise RuntimeError(
            f"node_feats {tuple(Xv.shape)} and edge_feats {tuple(Xe.shape)} must be V x h and E x h"
        )
    V, h = Xv.shape
    E = Xe.shape[0]
    if src.numel() != E:
        raise ValueError("src must have one entry per edge")
    ld = h if pitch is None else int(pitch)
    H0 = padded_rows(E, h, ld, Xv.dtype, dev)
    S = None
    if seg_ptr is not None:
        S = padded_rows(V, h, ld, Xv.dtype, dev)
    lib = _lib.load()
    _run(dev, lib.nt_dmpnn_init,
         _ptr(Xv), _ptr(Xe), _ptr(src), _ptr(seg_ptr), _ptr(perm), V, E, h, act[0], act[1],
         reduce_code(reduce), code, _ptr(H0), _ptr(S), _ptr(amax), 0 if ld == h else ld, int(skip_degree),
         _stream(dev))
    return H0, S


def _require_amax(amax: Tensor | None, dtype: torch.dtype, n: int = 2) -> None:
    if amax is None:
        return
    if dtype != torch.float32:
        raise ValueError("amax is fp32 only")
    if amax.dtype != torch.float32 or amax.numel() < n or not amax.is_contiguous():
        raise ValueError(f"amax must be a contiguous float32 device tensor of {n} elements")


def absmax(X: Tensor, out: Tensor | None = None) -> Tensor:
    """max |X| (fp32) into out[0] (a 1-element float32 device tensor, zero-filled if not given)."""
    dev = _require_device(X, out)
    _require_f32("X", X)
    if not X.is_contiguous():
        raise ValueError("absmax: X must be contiguous")
    if out is None:
        out = torch.zeros(1, dtype=torch.float32, device=dev)
    _run(dev, _lib.load().nt_absmax, _ptr(X), X.numel(), NT_F32, _ptr(out), _stream(dev))
    return out


def segment_reduce(
    X: Tensor,
    seg_ptr: Tensor,
    perm: Tensor | None,
    nseg: int,
    *,
    reduce: str = "sum",
    act: tuple[int, float] = (_lib.NT_ACT_IDENTITY, 0.0),
    out: Tensor | None = None,
) -> Tensor:
    """out[s] = reduce over rows X[perm[j]] (j in segment s) of act(row); empty segment -> 0."""
    dev = _require_device(X, seg_ptr, perm)
    code = _require_feat("X", X)
    if out is not None:
        _require_feat("out", out, X.dtype)
    if X.dim() != 2:
        raise ValueError("X must be 2-D")
    if seg_ptr.dtype != torch.int32 or seg_ptr.numel() != nseg + 1:
        raise ValueError("seg_ptr must be int32 of length nseg + 1")
    h = X.shape[1]
    if out is None:
        out = torch.empty(nseg, h, dtype=X.dtype, device=dev)
    if X.shape[0] == 0:  # no rows (an edge-free batch): every segment is empty -> 0 (torch_scatter)
        return out.zero_()
    lib = _lib.load()
    _run(dev, lib.nt_segment_reduce,
         _ptr(X), _ptr(seg_ptr), _ptr(perm), nseg, h, reduce_code(reduce), act[0], act[1], code,
         _ptr(out), _stream(dev))
    return out


def dmpnn_aggregate(H: Tensor, row_ptr: Tensor, perm: Tensor, V: int, *, reduce: str = "sum") -> Tensor:
    """S[v] = reduce over v's in-edges of relu(H[e]) (chemprop.py:36-39) through nt_dmpnn_aggregate
    (the dst CSR of nt_csr_build: row_ptr int32[V+1], perm int32[E])."""
    dev = _require_device(H, row_ptr, perm)
    code = _require_feat("H", H)
    if H.dim() != 2:
        raise ValueError("H must be 2-D")
    if row_ptr.dtype != torch.int32 or row_ptr.numel() != V + 1 or not row_ptr.is_contiguous():
        raise ValueError("row_ptr must be contiguous int32 of length V + 1")
    if perm.dtype != torch.int32 or perm.numel() != H.shape[0] or not perm.is_contiguous():
        raise ValueError("perm must be contiguous int32 with one entry per row of H")
    S = torch.empty(V, H.shape[1], dtype=H.dtype, device=dev)
    if H.shape[0] == 0:
        return S.zero_()
    _run(dev, _lib.load().nt_dmpnn_aggregate,
         _ptr(H), _ptr(row_ptr), _ptr(perm), V, H.shape[1], reduce_code(reduce), code, _ptr(S), _stream(dev))
    return S


CHUNK_ROWS = 32  # rows per chunk of the load-balanced segment reduce


def chunk_plan(seg_ptr: Tensor, chunk: int = CHUNK_ROWS) -> tuple:
    """(chunk_pos[nchunks+1], nchunks, chunk_ptr[nseg+1], chunk_seg[nchunks], comb_seg[ncomb]) for
    nt_segment_reduce_chunked: every segment cut into chunks of at most ``chunk`` CSR positions;
    chunk_seg[k] = the segment of chunk k when it is that segment's only chunk (pass 1 stores its
    result directly), else -1; comb_seg = the segments with != 1 chunk (pass 2's list).  Device ops;
    one host sync (the two counts)."""
    _require_device(seg_ptr)
    dev = seg_ptr.device
    sp = seg_ptr.to(torch.int64)
    n = sp[1:] - sp[:-1]
    nch = (n + chunk - 1) // chunk
    chunk_ptr64 = torch.zeros(n.numel() + 1, dtype=torch.int64, device=dev)
    torch.cumsum(nch, 0, out=chunk_ptr64[1:])
    multi = nch != 1
    nchunks, ncomb = (int(x) for x in torch.stack([chunk_ptr64[-1], multi.sum()]).tolist())
    seg_of = torch.repeat_interleave(torch.arange(n.numel(), device=dev), nch, output_size=nchunks)
    k_in_seg = torch.arange(nchunks, device=dev) - chunk_ptr64[seg_of]
    chunk_pos = torch.empty(nchunks + 1, dtype=torch.int32, device=dev)
    chunk_pos[:nchunks] = (sp[seg_of] + k_in_seg * chunk).to(torch.int32)
    chunk_pos[nchunks] = seg_ptr[-1]
    chunk_seg = torch.where(multi[seg_of], -1, seg_of).to(torch.int32)
    comb_seg = torch.nonzero(multi).flatten().to(torch.int32)
    assert comb_seg.numel() == ncomb
    return chunk_pos, nchunks, chunk_ptr64.to(torch.int32), chunk_seg, comb_seg


def _chunk_args(plan, nseg: int):
    """ctypes arguments (chunk_pos, nchunks, chunk_ptr, chunk_seg, comb_seg, ncomb) of a chunk plan."""
    if len(plan) != 5:
        raise ValueError("plan must be chunk_plan(seg_ptr): (chunk_pos, nchunks, chunk_ptr, chunk_seg, comb_seg)")
    chunk_pos, nchunks, chunk_ptr, chunk_seg, comb_seg = plan
    for name, t in (("chunk_pos", chunk_pos), ("chunk_ptr", chunk_ptr), ("chunk_seg", chunk_seg),
                    ("comb_seg", comb_seg)):
        if t.dtype != torch.int32:
            raise TypeError(f"{name} must be int32")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
    if (chunk_pos.numel() != nchunks + 1 or chunk_ptr.numel() != nseg + 1 or chunk_seg.numel() != nchunks
            or comb_seg.numel() > nseg):
        raise ValueError("plan must be chunk_plan(seg_ptr) of this CSR")
    return _ptr(chunk_pos), nchunks, _ptr(chunk_ptr), _ptr(chunk_seg), _ptr(comb_seg), comb_seg.numel()


def segment_reduce_chunked(
    X: Tensor,
    seg_ptr: Tensor,
    perm: Tensor | None,
    nseg: int,
    plan: tuple[Tensor, int, Tensor],
    *,
    reduce: str = "sum",
    act: tuple[int, float] = (_lib.NT_ACT_IDENTITY, 0.0),
    out: Tensor | None = None,
    amax: Tensor | None = None,
) -> Tensor:
    """segment_reduce load-balanced over chunks (plan = chunk_plan(seg_ptr)) for skewed segments;
    fp32: amax (1 zero-filled device float, optional) is raised to max|out|."""
    dev = _require_device(X, seg_ptr, perm, amax)
    code = _require_feat("X", X)
    if seg_ptr.dtype != torch.int32 or seg_ptr.numel() != nseg + 1:
        raise ValueError("seg_ptr must be int32 of length nseg + 1")
    cargs = _chunk_args(plan, nseg)
    nchunks = plan[1]
    h = X.shape[1]
    if out is None:
        out = torch.empty(nseg, h, dtype=X.dtype, device=dev)
    else:
        _require_feat("out", out, X.dtype)
    partial = torch.empty(max(nchunks, 1), h, dtype=torch.float32, device=dev)
    _run(dev, _lib.load().nt_segment_reduce_chunked,
         _ptr(X), _ptr(perm), *cargs, _ptr(seg_ptr), nseg, h,
         reduce_code(reduce), act[0], act[1], code, _ptr(partial), _ptr(out), _ptr(amax), _stream(dev))
    return out


def dmpnn_init_chunked(
    Xv: Tensor,
    Xe: Tensor,
    src: Tensor,
    seg_ptr: Tensor,
    perm: Tensor,
    plan: tuple[Tensor, int, Tensor],
    *,
    act: tuple[int, float] = (_lib.NT_ACT_IDENTITY, 0.0),
    reduce: str = "sum",
    amax: Tensor | None = None,
    pitch: int | None = None,
    H0: Tensor | None = None,
    S: Tensor | None = None,
    chunk_ids: Tensor | None = None,
) -> tuple[Tensor, Tensor]:
    """(H0, S) = dmpnn_init with layer 0's aggregation over the chunk plan of a hub graph (fp32,
    plan = chunk_plan(seg_ptr)): H0 written once, S combined from per-chunk partials.  amax (2
    zero-filled device floats, optional) raised to max|H0|, max|S|.  pitch: H0 and S as row-padded
    views (as dmpnn_init's)."""
    nchunks = plan[1]
    dev = _require_device(Xv, Xe, src, seg_ptr, perm, plan[0], plan[2], amax)
    if Xv.dtype != torch.float32 or Xe.dtype != torch.float32:
        raise ValueError("dmpnn_init_chunked is fp32 only")
    _require_amax(amax, Xv.dtype)
    _require_i64("src", src)
    for name, t in (("seg_ptr", seg_ptr), ("perm", perm)):
        if t.dtype != torch.int32:
            raise TypeError(f"{name} must be int32")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
    V, h = Xv.shape
    E = Xe.shape[0]
    if Xe.shape[1] != h or src.numel() != E or perm.numel() != E or seg_ptr.numel() != V + 1:
        raise ValueError("shape mismatch between Xv, Xe, src and the dst CSR")
    cargs = _chunk_args(plan, V)
    ld = h if pitch is None else int(pitch)
    if H0 is None:
        H0 = padded_rows(E, h, ld, torch.float32, dev)
    if S is None:
        S = padded_rows(V, h, ld, torch.float32, dev)
    if H0.shape != (E, h) or S.shape != (V, h) or _row_pitch("H0", H0) != ld or _row_pitch("S", S) != ld:
        raise ValueError("H0 / S must be E x h / V x h with the given row pitch")
    if chunk_ids is not None and (chunk_ids.dtype != torch.int32 or not chunk_ids.is_contiguous()
                                  or chunk_ids.numel() > nchunks):
        raise ValueError("chunk_ids must be contiguous int32 chunk indices of the plan")
    partial = torch.empty(max(nchunks, 1), h, dtype=torch.float32, device=dev)
    _run(dev, _lib.load().nt_dmpnn_init_chunked,
         _ptr(Xv.contiguous()), _ptr(Xe.contiguous()), _ptr(src), _ptr(perm), *cargs, _ptr(seg_ptr), V, E, h, act[0], act[1], reduce_code(reduce), _DTYPE_CODES[torch.float32],
         _ptr(partial), _ptr(H0), _ptr(S), _ptr(amax), 0 if ld == h else ld, _ptr(chunk_ids),
         0 if chunk_ids is None else chunk_ids.numel(), _stream(dev))
    return H0, S


def packed_weight_numel(h: int, dtype: torch.dtype = torch.float32) -> int:
    """Size (in 4-byte words) of one layer's packed weight image for feature dtype ``dtype``."""
    return _lib.load().nt_dmpnn_packed_weight_bytes(h, _DTYPE_CODES[dtype]) // 4


def pack_weights(W: Tensor, *, fk_only: bool = False) -> Tensor:
    """Pack one nn.Linear weight [h, h] (or a stack [L, h, h]) into the MFMA fragment image of its
    dtype (fp32: the two-part fp16 image of the fp32 layer kernel plus the older bf16-split images;
    bf16: one bf16 fragment image).  The image is an opaque float32-typed buffer.  fk_only (fp32):
    only the part nt_dmpnn_update_fused / dense_matmul read (nt_dmpnn_pack_weight_fk)."""
    dev = _require_device(W)
    code = _require_feat("weight", W)
    if W.dim() == 2:
        W3 = W.unsqueeze(0)
    else:
        W3 = W
    L, h, h2 = W3.shape
    if h != h2:
        raise ValueError(f"ChempropLayer weight must be square, got {tuple(W.shape)}")
    Wp = torch.empty(L, packed_weight_numel(h, W.dtype), dtype=torch.float32, device=dev)
    lib = _lib.load()
    if fk_only and W.dtype == torch.float32:
        W3 = W3.contiguous()
        _run(dev, lib.nt_dmpnn_pack_weight_fk, _ptr(W3), L, h, _ptr(Wp), _stream(dev))
    else:
        _run(dev, lib.nt_dmpnn_pack_weight, _ptr(W3), L, h, code, _ptr(Wp), _stream(dev))
    return Wp[0] if W.dim() == 2 else Wp


def pack_weights_fk_multi(Ws: Sequence[Tensor], with_t: bool = False) -> tuple[list[Tensor], list[Tensor] | None]:
    """fp32: the fk images (nt_dmpnn_pack_weight_fk's part of pack_weights) of up to 16 separate h x h
    weights and, with ``with_t``, of their transposes (the backward's dA image), in one launch pair
    (nt_dmpnn_pack_weights_fk).  Bytes equal pack_weights(W, fk_only=True) and
    pack_weights(W.t().contiguous(), fk_only=True)."""
    if not Ws:
        return [], ([] if with_t else None)
    dev = _require_device(*Ws)
    h = Ws[0].shape[0]
    for W in Ws:
        _require_f32("weight", W)
        if W.shape != (h, h) or not W.is_contiguous():
            raise ValueError("pack_weights_fk_multi: contiguous h x h weights of one hidden size")
    if len(Ws) > 16:
        raise ValueError("pack_weights_fk_multi: at most 16 weights per call")
    n = packed_weight_numel(h, torch.float32)
    imgs = [torch.empty(n, dtype=torch.float32, device=dev) for _ in Ws]
    imgsT = [torch.empty(n, dtype=torch.float32, device=dev) for _ in Ws] if with_t else None
    arr = ctypes.c_void_p * len(Ws)
    _run(dev, _lib.load().nt_dmpnn_pack_weights_fk, arr(*[W.data_ptr() for W in Ws]), len(Ws), h,
         arr(*[t.data_ptr() for t in imgs]), None if imgsT is None else arr(*[t.data_ptr() for t in imgsT]),
         _stream(dev))
    return imgs, imgsT


def dmpnn_update(
    H: Tensor,
    S: Tensor,
    src: Tensor,
    rev: Tensor,
    Wp: Tensor,
    bias: Tensor | None,
    *,
    residual: bool = True,
    act: tuple[int, float] = (_lib.NT_ACT_RELU, 0.0),
    out: Tensor | None = None,
) -> Tensor:
    """H_out = (residual ? H : 0) + (S[src] - act(H[rev])) @ W^T + b   (one fused launch)."""
    dev = _require_device(H, S, src, rev, Wp, bias, out)
    code = _require_feat("H", H)
    _require_feat("S", S, H.dtype)
    _require_i64("src", src)
    _require_i64("rev_index", rev)
    E, h = H.shape
    V = S.shape[0]
    if S.shape[1] != h or src.numel() != E or rev.numel() != E:
        raise ValueError("shape mismatch between H, S, src and rev_index")
    if Wp.numel() != packed_weight_numel(h, H.dtype):
        raise ValueError(f"Wp is not a packed {H.dtype} weight image for this hidden size")
    if bias is not None:
        _require_feat("bias", bias, H.dtype)
        if bias.numel() != h:
            raise ValueError("bias must have h entries")
    if out is None:
        out = torch.empty_like(H)
    else:
        _require_feat("out", out, H.dtype)
    lib = _lib.load()
    # fp32 split scales: a 2-float device workspace owned by the caller (ABI 6), allocated on the
    # current stream by the caching allocator, so its reuse is stream-ordered
    ws = torch.empty(2, dtype=torch.float32, device=dev) if code == NT_F32 and h % 4 == 0 else None
    _run(dev, lib.nt_dmpnn_update,
         _ptr(H), _ptr(S), _ptr(src), _ptr(rev), _ptr(Wp), _ptr(bias), V, E, h, int(residual),
         act[0], act[1], code, _ptr(ws), _ptr(out), _stream(dev))
    return out


def fused_supported(V: int, E: int, h: int, dtype: torch.dtype = torch.float32) -> bool:
    """Shapes nt_dmpnn_update_fused accepts: the fp32 fk kernel (h % 4 == 0, h <= 8192) or the bf16
    tile kernel (h % 8 == 0, h <= 512)."""
    if dtype == torch.bfloat16:
        return h % 8 == 0 and 8 <= h <= 512 and E < 2**31
    return (dtype == torch.float32 and h % 4 == 0 and 4 <= h <= 8192 and E * h // 4 < 2**31
            and V * h // 4 < 2**31 and E < 2**31 and V < 2**31)


PLAN_NCU = 256  # CUs the balanced tile plans are cut for (MI355X; host and device plans agree)
# slots the 64-row plans are balanced over.  Their kernels run two workgroups per CU, but balancing
# for 512 workgroups (~51-row tiles) measured slower than for the 256 CUs (~61 rows, whose tile count
# leaves some workgroups one tile short): config 2 layer 118-119 vs 107-110 us, config 3 233-235 vs
# 228 us, training 1.545 vs 1.478-1.495 ms (tools/r6_slots.sh, profiles/r6/slots_ab.txt)
PLAN_SLOTS64 = PLAN_NCU


def fused_tile_rows(h: int, dtype: torch.dtype, act: tuple[int, float] = (_lib.NT_ACT_RELU, 0.0),
                    reduce: str = "sum", agg_act: tuple[int, float] = (_lib.NT_ACT_RELU, 0.0)) -> int:
    """Row capacity of a nt_dmpnn_update_fused tile for this layer (128 or 64)."""
    code = NT_BF16 if dtype == torch.bfloat16 else NT_F32
    return int(_lib.load().nt_dmpnn_fused_tile_rows(h, code, act[0], reduce_code(reduce), agg_act[0]))


def tile_stride(E: int, max_in_degree: int, rows: int, ncu: int = PLAN_NCU) -> int:
    """Stride of the tile plan with tiles of at most `rows` rows, balanced over ncu CUs."""
    return int(_lib.load().nt_dmpnn_tile_stride(E, max_in_degree, rows, ncu))


def tile_plan(dst_ptr: Tensor, E: int, max_in_degree: int, rows: int = 64,
              ncu: int = 0, hub_degree: int = 0) -> tuple[Tensor, int, Tensor]:
    """(tile_ptr[ntiles+1], ntiles, dst_sorted[E]) for nt_dmpnn_update_fused: node-aligned tiles of
    at most `rows` rows (max_in_degree <= 32), balanced to whole rounds of ncu tiles (ncu = 0: the
    largest tiles; the engine's 128-row plans use PLAN_NCU).  hub_degree > 0: nodes with more
    in-edges are hubs, cut at the stride (nt_dmpnn_tile_plan_hubs; max_in_degree is then the largest
    non-hub in-degree).  The plan's largest tile is checked against `rows` here, where the plan is
    built (one device->host read per plan; the engine builds one per graph layout): the layer kernels
    clamp a larger tile and keep no status word, so a wrong max_in_degree must fail at this call."""
    dev = _require_device(dst_ptr)
    if dst_ptr.dtype != torch.int32:
        raise TypeError("dst_ptr must be int32")
    V = dst_ptr.numel() - 1
    lib = _lib.load()
    stride = tile_stride(E, max_in_degree, rows, ncu) if E > 0 else 1
    if E > 0 and stride <= 0:
        raise ValueError(f"max in-degree {max_in_degree} exceeds the tile rows {rows}")
    ntiles = int(lib.nt_dmpnn_tile_count(E, stride))
    tile_ptr = torch.empty(ntiles + 1, dtype=torch.int32, device=dev)
    dsts = torch.empty(max(E, 1), dtype=torch.int32, device=dev)[:E]
    if hub_degree > 0:
        _run(dev, lib.nt_dmpnn_tile_plan_hubs,
             _ptr(dst_ptr), V, E, stride, int(hub_degree), _ptr(tile_ptr), ntiles, _ptr(dsts), _stream(dev))
    else:
        _run(dev, lib.nt_dmpnn_tile_plan,
             _ptr(dst_ptr), V, E, stride, _ptr(tile_ptr), ntiles, _ptr(dsts), _stream(dev))
    if ntiles > 0:
        mx = int((tile_ptr[1:] - tile_ptr[:-1]).max())
        if mx > rows:
            raise ValueError(f"tile plan holds a tile of {mx} rows > {rows}: max_in_degree={max_in_degree} is "
                             "below the graph's largest (non-hub) in-degree")
    return tile_ptr, ntiles, dsts


def hub_runs(row_table: Tensor, dst_ptr: Tensor, dst_sorted: Tensor, tile_ptr: Tensor, hub_degree: int,
             run_rows: int) -> tuple[Tensor, int, Tensor, Tensor]:
    """A row table whose hub rows (nodes with more than hub_degree in-edges) are sub-runs for the fused
    layer's hub partials: runs of one hub's consecutive positions within a tile (tile_ptr), cut every
    run_rows rows (<= the launch's max_in_degree, so the kernel's segmented scan covers them), entry
    w = -((slot << 2) | start | end << 1) - 1.  Returns (table, nslots, hubs, slot_ptr) for
    dmpnn_update_fused(S_part=...) and hub_combine.  Device ops; one sync (the slot count)."""
    dev = _require_device(row_table, dst_ptr, dst_sorted, tile_ptr)
    E, V = row_table.shape[0], dst_ptr.numel() - 1
    run_rows = max(1, int(run_rows))
    dp = dst_ptr.long()
    deg = dp[1:] - dp[:-1]
    is_hub = deg > hub_degree
    d = dst_sorted.long()
    pos = torch.arange(E, device=dev)
    hub_row = is_hub[d]
    ts = torch.zeros(E + 1, dtype=torch.bool, device=dev)
    ts[tile_ptr.long()] = True
    run_start = hub_row & ((pos == dp[d]) | ts[:E])
    run_end = hub_row & ((pos + 1 == dp[d + 1]) | ts[1:])
    # offset of each row in its run (the run's start position by a running max), cut every run_rows
    rs = torch.cummax(torch.where(run_start, pos, torch.zeros_like(pos)), 0).values
    off = pos - rs
    sub_start = hub_row & (off % run_rows == 0)
    sub_end = hub_row & ((off % run_rows == run_rows - 1) | run_end)
    slot = torch.cumsum(sub_start.long(), 0) - 1
    hubs = torch.nonzero(is_hub).flatten()
    nslots = int(sub_start.sum()) if E else 0
    w = -(((slot << 2) | sub_start.long() | (sub_end.long() << 1))) - 1
    out = row_table.clone()
    out[:, 3] = torch.where(hub_row, w, row_table[:, 3].long()).to(torch.int32)
    # slot_ptr[v] = sub-runs starting before node v's first position (the hubs' slot CSR)
    before = torch.zeros(E + 1, dtype=torch.long, device=dev)
    torch.cumsum(sub_start.long(), 0, out=before[1:])
    slot_ptr = before[dp].to(torch.int32)
    return out, nslots, hubs.to(torch.int32), slot_ptr


def hub_combine(partial: Tensor, hubs: Tensor, slot_ptr: Tensor, seg_ptr: Tensor, out: Tensor, *,
                reduce: str = "sum", amax: Tensor | None = None) -> Tensor:
    """out[v] = reduce over the partial rows [slot_ptr[v], slot_ptr[v + 1]) for v in hubs
    (nt_dmpnn_hub_combine); out may be a row-padded view."""
    dev = _require_device(partial, hubs, slot_ptr, seg_ptr, out, amax)
    if partial.dtype != torch.float32 or out.dtype != torch.float32 or not partial.is_contiguous():
        raise TypeError("hub_combine: contiguous fp32 partial rows, fp32 out")
    V = seg_ptr.numel() - 1
    if slot_ptr.numel() != V + 1 or out.shape[0] != V:
        raise ValueError("slot_ptr must have V + 1 entries and out V rows")
    ld = _row_pitch("out", out)
    h = out.shape[1]
    _run(dev, _lib.load().nt_dmpnn_hub_combine, _ptr(partial), _ptr(hubs), _ptr(slot_ptr), hubs.numel(),
         _ptr(seg_ptr), V, h, reduce_code(reduce), NT_F32, _ptr(amax), _ptr(out), 0 if ld == h else ld, _stream(dev))
    return out


def mark_hub_rows(row_table: Tensor, dst_ptr: Tensor, hub_degree: int) -> Tensor:
    """In place: the row-table entries of nodes with more than hub_degree in-edges lose their
    "last in-edge" flag (nt_dmpnn_mark_hub_rows), so the fused layer leaves their S_out rows to
    hub_aggregate."""
    dev = _require_device(row_table, dst_ptr)
    if dst_ptr.dtype != torch.int32:
        raise TypeError("dst_ptr must be int32")
    _run(dev, _lib.load().nt_dmpnn_mark_hub_rows, _ptr(row_table), row_table.shape[0], _ptr(dst_ptr),
         dst_ptr.numel() - 1, int(hub_degree), _stream(dev))
    return row_table


def hub_aggregate(X: Tensor, perm: Tensor, seg_ptr: Tensor, hubs: Tensor, out: Tensor, *, reduce: str = "sum",
                  act: tuple[int, float] = (_lib.NT_ACT_IDENTITY, 0.0), amax: Tensor | None = None) -> Tensor:
    """out[v] = reduce over the in-edges p of v of act(X[perm[p]]) for the nodes v in ``hubs`` (int32),
    other rows of ``out`` untouched; amax (1 float, may be None) raised to max|out[hubs]|.  X and out
    may be row-padded views of one common pitch."""
    dev = _require_device(X, perm, seg_ptr, hubs, out, amax)
    if X.dtype != torch.float32 or out.dtype != torch.float32:
        raise TypeError("hub_aggregate is fp32 only")
    ld = _row_pitch("X", X)
    if _row_pitch("out", out) != ld:
        raise ValueError("X and out must share one row pitch")
    if hubs.dtype != torch.int32 or seg_ptr.dtype != torch.int32 or perm.dtype != torch.int32:
        raise TypeError("hubs, seg_ptr and perm must be int32")
    if out.shape[1] != X.shape[1] or out.shape[0] != seg_ptr.numel() - 1:
        raise ValueError("out must be nseg x h")
    _run(dev, _lib.load().nt_dmpnn_hub_aggregate, _ptr(X), _ptr(perm), _ptr(seg_ptr), _ptr(hubs), hubs.numel(),
         X.shape[1], reduce_code(reduce), act[0], act[1], NT_F32, _ptr(amax), _ptr(out),
         0 if ld == X.shape[1] else ld, _stream(dev))
    return out


def dmpnn_update_fused(
    H: Tensor,
    S: Tensor,
    src: Tensor,
    rev: Tensor,
    Wp: Tensor,
    bias: Tensor | None,
    *,
    residual: bool = True,
    act: tuple[int, float] = (_lib.NT_ACT_RELU, 0.0),
    plan: tuple[Tensor, int, Tensor] | None = None,
    tile_rows: int = 64,
    max_in_degree: int = 32,
    perm: Tensor | None = None,
    reduce: str = "sum",
    agg_act: tuple[int, float] = (_lib.NT_ACT_RELU, 0.0),
    zero_fill: bool = False,
    amax_in: Tensor | None = None,
    amax_out: Tensor | None = None,
    row_table: Tensor | None = None,
    out: Tensor | None = None,
    S_out: Tensor | None = None,
    pitch_out: int | None = None,
    S_part: Tensor | None = None,
    n_nodes: int | None = None,
) -> tuple[Tensor, Tensor | None]:
    """H_out = (residual ? H : 0) + (S[src] - act(H[rev])) @ W^T + b and, with a tile plan (tiles of at
    most ``tile_rows`` rows), S_out = scatter(agg_act(H_out), dst, reduce) in the same persistent launch.

    fp32: H and S may be row-padded views with one common pitch (see dmpnn_init's ``pitch``); H_out /
    S_out are allocated with rows ``pitch_out`` floats apart (default: dense), or given with one pitch.

    fp32: ``amax_in`` = (max|H|, max|S|) on the device (computed here with nt_absmax when not given);
    ``amax_out`` (2 zero-filled floats) receives max|H_out|, max|S_out| for the next layer.
    ``row_table`` (with a plan): nt_dmpnn_row_table of (perm, dst_sorted, src, rev), built here
    when not given (cache it per graph).
    ``zero_fill`` must be True when some node has no in-edge (its S_out row is then 0).
    ``S_part`` (fp32, slots x h): the hub partial rows when the row table marks hub sub-runs
    (hub_runs); hub_combine then finishes the hubs' S_out rows.
    ``n_nodes``: the aggregation's segment count, i.e. the rows S_out must hold (default: S's rows;
    the backward's fused dA passes S = G with E rows and S_out with the graph's V)."""
    dev = _require_device(H, S, src, rev, Wp, bias, out, S_out, perm, amax_in, amax_out)
    ld_in = _row_pitch("H", H)
    code = _DTYPE_CODES[H.dtype]
    if _row_pitch("S", S, H.dtype) != ld_in:
        raise ValueError("H and S must share one row pitch")
    _require_i64("src", src)
    _require_i64("rev_index", rev)
    _require_amax(amax_in, H.dtype)
    _require_amax(amax_out, H.dtype)
    E, h = H.shape
    V = S.shape[0]
    if S.shape[1] != h or src.numel() != E or rev.numel() != E:
        raise ValueError("shape mismatch between H, S, src and rev_index")
    if Wp.numel() != packed_weight_numel(h, H.dtype):
        raise ValueError(f"Wp is not a packed {H.dtype} weight image for this hidden size")
    if bias is not None:
        _require_feat("bias", bias, H.dtype)
        if bias.numel() != h:
            raise ValueError("bias must have h entries")
    if out is None:
        out = padded_rows(E, h, h if pitch_out is None else int(pitch_out), H.dtype, dev)
    ld_out = _row_pitch("out", out, H.dtype)
    tile_ptr = dsts = None
    ntiles = 0
    if plan is not None:
        tile_ptr, ntiles, dsts = plan
        if perm is None or perm.dtype != torch.int32 or perm.numel() != E:
            raise ValueError("fused aggregation needs the int32 dst CSR permutation")
        if dsts is None or dsts.dtype != torch.int32 or dsts.numel() != E:
            raise ValueError("the plan's dst_sorted must be int32 with E entries")
        n_out = V if n_nodes is None else int(n_nodes)
        if S_part is not None and (S_part.dtype != torch.float32 or not S_part.is_contiguous()
                                   or S_part.dim() != 2 or S_part.shape[1] != h or S_part.shape[0] < 1):
            raise ValueError("S_part must be a contiguous fp32 (slots x h) tensor")
        if S_out is None:
            S_out = padded_rows(n_out, h, ld_out, H.dtype, dev)
            if zero_fill:
                S_out.zero_()
        else:
            if _row_pitch("S_out", S_out, H.dtype) != ld_out:
                raise ValueError("out and S_out must share one row pitch")
            if S_out.shape[0] < n_out or S_out.shape[1] != h:
                raise ValueError(f"S_out must hold n_nodes={n_out} rows of h={h}")
            if zero_fill:
                S_out.zero_()
    else:
        perm = None
        S_out = None
        if S_part is not None:
            raise ValueError("S_part needs a tile plan")
    if plan is not None and row_table is None and E > 0:
        row_table = dmpnn_row_table(perm, dsts, src, rev, V)
    if H.dtype == torch.float32 and amax_in is None and E > 0:
        amax_in = torch.zeros(2, dtype=torch.float32, device=dev)
        absmax(H.contiguous(), amax_in[0:1])
        absmax(S.contiguous(), amax_in[1:2])
    lib = _lib.load()
    _run(dev, lib.nt_dmpnn_update_fused,
         _ptr(H), _ptr(S), _ptr(src), _ptr(rev), _ptr(Wp), _ptr(bias), V, E, h, int(residual),
         act[0], act[1], _ptr(tile_ptr), ntiles, int(tile_rows), int(max_in_degree), _ptr(perm), _ptr(dsts),
         _ptr(row_table), reduce_code(reduce), agg_act[0], agg_act[1], code, _ptr(amax_in), _ptr(amax_out),
         _ptr(out), _ptr(S_out), _ptr(S_part), 0 if ld_in == h else ld_in, 0 if ld_out == h else ld_out,
         _stream(dev))
    return out, S_out


def dmpnn_row_table(perm: Tensor, dst_sorted: Tensor, src: Tensor, rev: Tensor, V: int) -> Tensor:
    """E x 4 int32: {edge, src, rev, (node << 2) | start | end << 1} per dst-sorted position (the fp32
    layer kernel's one-load view of a fused plan's rows)."""
    dev = _require_device(perm, dst_sorted, src, rev)
    _require_i64("src", src)
    _require_i64("rev_index", rev)
    E = perm.numel()
    out = torch.empty(max(E, 1), 4, dtype=torch.int32, device=dev)[:E]
    _run(dev, _lib.load().nt_dmpnn_row_table, _ptr(perm), _ptr(dst_sorted), _ptr(src), _ptr(rev), V, E, _ptr(out),
         _stream(dev))
    return out


def dense_matmul(X: Tensor, Wp: Tensor, out: Tensor | None = None, *, kernel: str = "fk",
                 amax: Tensor | None = None) -> Tensor:
    """X @ W^T for the packed image Wp of W: the layer GEMM alone.  With Wp = pack_weights(W.t()) it is
    the backward's dA = G @ W.  fp32 (h % 4 == 0), kernel = "fk": the fp16x3 layer kernel in dense
    mode (amax: 2 device floats whose [1] >= max|X|, else nt_absmax first; any h); "pk": the bf16x6
    persistent kernel (h <= 304).  bf16 (h <= 512): the bf16 layer kernel without gathers (fp32
    accumulate, one rounding)."""
    dev = _require_device(X, Wp, out, amax)
    code = _require_feat("X", X)
    M, h = X.shape
    if Wp.numel() != packed_weight_numel(h, X.dtype):
        raise ValueError(f"Wp is not a packed {X.dtype} weight image for this hidden size")
    if out is None:
        out = torch.empty_like(X)
    if code == NT_BF16:
        if h > 512:
            raise ValueError("dense_matmul: bf16 needs h <= 512")
        _run(dev, _lib.load().nt_dmpnn_dense_matmul, _ptr(X), M, h, _ptr(Wp), NT_BF16, None, None, _ptr(out),
             _stream(dev))
        return out
    if kernel == "fk":
        if amax is None:
            amax = torch.zeros(2, dtype=torch.float32, device=dev)
            absmax(X, amax[1:2])
        else:
            _require_amax(amax, X.dtype)
    elif kernel != "pk":
        raise ValueError("kernel must be 'fk' or 'pk'")
    # kernel = "pk" passes no amax: the diagnostic library then runs the bf16x6 kernel, the shipping one
    # the fk kernel with max|X| written into this caller-owned workspace (ABI 6)
    ws = torch.empty(2, dtype=torch.float32, device=dev) if amax is None else None
    _run(dev, _lib.load().nt_dmpnn_dense_matmul, _ptr(X), M, h, _ptr(Wp), NT_F32, _ptr(amax), _ptr(ws), _ptr(out),
         _stream(dev))
    return out


def weight_grad(G: Tensor, H: Tensor | None, S: Tensor, src: Tensor | None, rev: Tensor | None, *,
                act: tuple[int, float] = (_lib.NT_ACT_RELU, 0.0), bias: bool = True,
                amax_G: Tensor | None = None, amax_HS: Tensor | None = None) -> tuple[Tensor, Tensor | None]:
    """(dW, db) = (G^T A, sum_e G[e]) with A[e] = S[src e] - act(H[rev e]) formed on the fly
    (src = rev = None: A = S).  Split-K, deterministic.  fp32: with amax_G (1 device float >= max|G|)
    and amax_HS (2 floats >= max|H|, max|S|), h <= 320 and src / rev given, the two-part fp16 kernel
    (nt_dmpnn_weight_grad_fk); else the bf16x6 kernel.  bf16 (h <= 512, even, src / rev given): A
    rounded to bf16 as the forward's message, one bf16 MFMA per tile; dW and db come back in fp32."""
    dev = _require_device(G, H, S, src, rev, amax_G, amax_HS)
    code = _require_feat("G", G)
    _require_feat("S", S, G.dtype)
    if code == NT_BF16 and (src is None or G.shape[1] > 512 or G.shape[1] % 2):
        raise ValueError("weight_grad: bf16 needs src / rev_index and an even h <= 512")
    E, h = G.shape
    if (src is None) != (rev is None):
        raise ValueError("weight_grad: pass both src and rev_index or neither")
    if src is not None:
        assert H is not None
        _require_feat("H", H, G.dtype)
        _require_i64("src", src)
        _require_i64("rev_index", rev)
        if H.shape != (E, h) or S.shape[1] != h or src.numel() != E or rev.numel() != E:
            raise ValueError("shape mismatch between G, H, S, src and rev_index")
    elif S.shape != (E, h):
        raise ValueError("weight_grad: S must be E x h when src is None")
    for n_, t in (("G", G), ("H", H), ("S", S)):
        if t is not None and not t.is_contiguous():
            raise ValueError(f"weight_grad: {n_} must be contiguous")
    lib = _lib.load()
    # the workspace is sized by the plan of the launch device (its CU count): query under its guard
    if dev.index is not None and dev.index != torch.cuda.current_device():
        with torch.cuda.device(dev):
            nbytes = lib.nt_dmpnn_weight_grad_workspace(E, h)
    else:
        nbytes = lib.nt_dmpnn_weight_grad_workspace(E, h)
    if nbytes < 0:
        raise ValueError(f"weight_grad: bad sizes E={E} h={h}")
    ws = torch.empty((max(nbytes, 4) + 3) // 4, dtype=torch.float32, device=dev)
    dW = torch.empty(h, h, dtype=torch.float32, device=dev)
    db = torch.empty(h, dtype=torch.float32, device=dev) if bias else None
    if code == NT_F32 and amax_G is not None and amax_HS is not None and src is not None and h <= 320:
        _require_amax(amax_G, G.dtype, n=1)
        _require_amax(amax_HS, G.dtype)
        _run(dev, lib.nt_dmpnn_weight_grad_fk, _ptr(G), _ptr(H), _ptr(S), _ptr(src), _ptr(rev), S.shape[0], E,
             h, act[0], act[1], _ptr(amax_G), _ptr(amax_HS), NT_F32, _ptr(ws), ws.numel() * 4, _ptr(dW), _ptr(db),
             _stream(dev))
        return dW, db
    _run(dev, lib.nt_dmpnn_weight_grad, _ptr(G), _ptr(H), _ptr(S), _ptr(src), _ptr(rev), S.shape[0], E, h,
         act[0], act[1], code, _ptr(ws), ws.numel() * 4, _ptr(dW), _ptr(db), _stream(dev))
    return dW, db


def segment_arg(X: Tensor, seg_ptr: Tensor, perm: Tensor | None, nseg: int, reduce: str, *,
                act: tuple[int, float] = (_lib.NT_ACT_IDENTITY, 0.0)) -> Tensor:
    """int32 (nseg x h): the first row (ascending CSR order) of each segment holding the max / min
    of act(X) per column, -1 for empty segments (torch_scatter scatter_max / scatter_min's arg).
    fp32 or bf16 X."""
    dev = _require_device(X, seg_ptr, perm)
    code = _require_feat("X", X)
    if reduce not in ("max", "min"):
        raise ValueError("segment_arg: reduce must be 'max' or 'min'")
    h = X.shape[1]
    arg = torch.empty(nseg, h, dtype=torch.int32, device=dev)
    if X.shape[0] == 0:  # no rows: every segment is empty
        return arg.fill_(-1)
    _run(dev, _lib.load().nt_segment_arg, _ptr(X), _ptr(seg_ptr), _ptr(perm), nseg, h, reduce_code(reduce),
         act[0], act[1], code, _ptr(arg), _stream(dev))
    return arg


def dmpnn_edge_backward_arg(G: Tensor | None, H: Tensor, dA: Tensor, dS: Tensor, arg: Tensor, dst: Tensor,
                            rev_ptr: Tensor, rev_perm: Tensor, *, residual: bool = True,
                            act: tuple[int, float] = (_lib.NT_ACT_RELU, 0.0), amax: Tensor | None = None) -> Tensor:
    """dL/dH_l for a max / min aggregation (arg = segment_arg of act(H_l) over the dst CSR); amax (1
    zero-filled device float, optional, fp32 only) is raised to max|out|.  fp32 or bf16 storage."""
    dev = _require_device(G, H, dA, dS, arg, dst, rev_ptr, rev_perm, amax)
    code = _require_feat("H", H)
    for n_, t in (("dA", dA), ("dS", dS)) + ((("G", G),) if G is not None else ()):
        _require_feat(n_, t, H.dtype)
    if amax is not None and code != NT_F32:
        raise ValueError("amax is fp32 only")
    E, h = H.shape
    V = dS.shape[0]
    out = torch.empty_like(H)
    _run(dev, _lib.load().nt_dmpnn_edge_backward_arg, _ptr(G), _ptr(H), _ptr(dA), _ptr(dS), _ptr(arg),
         _ptr(dst), _ptr(rev_ptr), _ptr(rev_perm), V, E, h, int(residual), act[0], act[1], code,
         _ptr(out), _ptr(amax), _stream(dev))
    return out


def gather_rows_arg(X: Tensor, idx: Tensor, arg: Tensor, *, base: Tensor | None = None,
                    amax: Tensor | None = None) -> Tensor:
    """out[i] = base[i] + (arg[idx i] == i ? X[idx i] : 0) (max / min scatter backward); amax as
    dmpnn_edge_backward_arg.  fp32 or bf16."""
    dev = _require_device(X, idx, arg, base, amax)
    code = _require_feat("X", X)
    if base is not None:
        _require_feat("base", base, X.dtype)
    if amax is not None and code != NT_F32:
        raise ValueError("amax is fp32 only")
    n, h = idx.numel(), X.shape[1]
    out = torch.empty(n, h, dtype=X.dtype, device=dev)
    _run(dev, _lib.load().nt_gather_rows_arg, _ptr(base), _ptr(X), _ptr(idx), _ptr(arg), n, h, code,
         _ptr(out), _ptr(amax), _stream(dev))
    return out


# ------------------------------------------------------------------------------------ backward
def dmpnn_message(H: Tensor, S: Tensor, src: Tensor, rev: Tensor, *,
                  act: tuple[int, float] = (_lib.NT_ACT_RELU, 0.0), out: Tensor | None = None) -> Tensor:
    """A = S[src] - act(H[rev])  (the layer message, recomputed for the weight gradient)."""
    dev = _require_device(H, S, src, rev, out)
    code = _require_feat("H", H)
    _require_feat("S", S, H.dtype)
    _require_i64("src", src)
    _require_i64("rev_index", rev)
    E, h = H.shape
    V = S.shape[0]
    if S.shape[1] != h or src.numel() != E or rev.numel() != E:
        raise ValueError("shape mismatch between H, S, src and rev_index")
    if out is None:
        out = torch.empty_like(H)
    else:
        _require_feat("out", out, H.dtype)
    _run(dev, _lib.load().nt_dmpnn_message,
         _ptr(H), _ptr(S), _ptr(src), _ptr(rev), V, E, h, act[0], act[1], code, _ptr(out), _stream(dev))
    return out


def dmpnn_edge_backward(G: Tensor | None, H: Tensor, dA: Tensor, dS: Tensor, dst: Tensor,
                        rev_ptr: Tensor, rev_perm: Tensor, dst_ptr: Tensor | None, *,
                        residual: bool = True, act: tuple[int, float] = (_lib.NT_ACT_RELU, 0.0),
                        reduce: str = "sum", out: Tensor | None = None, amax: Tensor | None = None) -> Tensor:
    """dL/dH_l = (residual ? G : 0) + act'(H) * (dS[dst] / c - scatter(dA, rev))  (see header); fp32:
    amax (1 zero-filled device float, optional) is raised to max|out|."""
    dev = _require_device(G, H, dA, dS, dst, rev_ptr, rev_perm, dst_ptr, out, amax)
    code = _require_feat("H", H)
    for name, t in (("dA", dA), ("dS", dS)):
        _require_feat(name, t, H.dtype)
    if residual:
        if G is None:
            raise ValueError("residual backward needs G")
        _require_feat("G", G, H.dtype)
    _require_i64("dst", dst)
    E, h = H.shape
    V = dS.shape[0]
    if dA.shape != H.shape or dS.shape[1] != h or dst.numel() != E or rev_ptr.numel() != E + 1:
        raise ValueError("shape mismatch in dmpnn_edge_backward")
    if reduce == "mean" and dst_ptr is None:
        raise ValueError("mean reduce needs the dst CSR")
    if out is None:
        out = torch.empty_like(H)
    else:
        _require_feat("out", out, H.dtype)
    _run(dev, _lib.load().nt_dmpnn_edge_backward,
         _ptr(G if residual else None), _ptr(H), _ptr(dA), _ptr(dS), _ptr(dst), _ptr(rev_ptr),
         _ptr(rev_perm), _ptr(dst_ptr), V, E, h, int(residual), act[0], act[1], reduce_code(reduce),
         code, _ptr(out), _ptr(amax), _stream(dev))
    return out


def gather_rows(X: Tensor, idx: Tensor, *, base: Tensor | None = None, seg_ptr: Tensor | None = None,
                out: Tensor | None = None, amax: Tensor | None = None) -> Tensor:
    """out[i] = (base[i] if base is given) + X[idx[i]], divided by max(segment size of idx[i], 1)
    when ``seg_ptr`` is given (the backward of a mean scatter); fp32: amax as dmpnn_edge_backward."""
    dev = _require_device(X, idx, base, seg_ptr, out, amax)
    code = _require_feat("X", X)
    _require_i64("idx", idx)
    nseg, h = X.shape
    n = idx.numel()
    if base is not None:
        _require_feat("base", base, X.dtype)
        if base.shape != (n, h):
            raise ValueError("base must be n x h")
    if seg_ptr is not None and (seg_ptr.dtype != torch.int32 or seg_ptr.numel() != nseg + 1):
        raise ValueError("seg_ptr must be int32 of length nseg + 1")
    if out is None:
        out = torch.empty(n, h, dtype=X.dtype, device=dev)
    else:
        _require_feat("out", out, X.dtype)
    _run(dev, _lib.load().nt_gather_rows,
         _ptr(base), _ptr(X), _ptr(idx), _ptr(seg_ptr), n, nseg, h, code, _ptr(out), _ptr(amax), _stream(dev))
    return out


# ------------------------------------------------------------------------------------ embedding
def _check_types(name: str, idx: Tensor, num_types: int) -> None:
    _require_i64(name, idx)
    if idx.dim() != 2:
        raise ValueError(f"{name} must be n x k type indices")
    if idx.numel():
        mm = torch.stack([idx.min(), idx.max()]).cpu()
        if mm[0] < 0 or mm[1] >= num_types:
            raise IndexError(f"{name}: type index out of range for an embedding of {num_types} rows")


def embed_bag(table: Tensor, idx: Tensor, *, validate: bool = True, out: Tensor | None = None) -> Tensor:
    """nn.EmbeddingBag(mode="sum") of an n x k index matrix: out[i] = sum_j table[idx[i, j]]."""
    dev = _require_device(table, idx, out)
    code = _require_feat("table", table)
    ntypes, h = table.shape
    if validate:
        _check_types("idx", idx, ntypes)
    else:
        _require_i64("idx", idx)
    n, k = idx.shape
    if out is None:
        out = torch.empty(n, h, dtype=table.dtype, device=dev)
    _run(dev, _lib.load().nt_embed_bag,
         _ptr(table), ntypes, _ptr(idx), n, k, h, code, _ptr(out), _stream(dev))
    return out


def dmpnn_init_embed(
    node_table: Tensor,
    node_types: Tensor,
    edge_table: Tensor,
    edge_types: Tensor,
    src: Tensor,
    seg_ptr: Tensor | None = None,
    perm: Tensor | None = None,
    *,
    act: tuple[int, float] = (_lib.NT_ACT_RELU, 0.0),
    reduce: str = "sum",
    validate: bool = True,
    amax: Tensor | None = None,
    pitch: int | None = None,
    records: Tensor | None = None,
) -> tuple[Tensor, Tensor | None]:
    """H0 = Xv[src] + Xe with Xv = EmbeddingBag(node_table)(node_types), Xe likewise, never
    materialised; optionally fused with S = scatter(act(H0), dst) (needs the dst CSR).
    amax (fp32, 2 zero-filled device floats): raised to max|H0|, max|S|.
    records: embed_edge_records of this graph (fp32 with S, 7 + 2 type columns): the wave-per-node
    init over them (same bits)."""
    dev = _require_device(node_table, node_types, edge_table, edge_types, src, seg_ptr, perm, amax, records)
    _require_amax(amax, node_table.dtype)
    code = _require_feat("node_table", node_table)
    _require_feat("edge_table", edge_table, node_table.dtype)
    if node_table.shape[1] != edge_table.shape[1]:
        raise RuntimeError("node and edge embedding tables must share the hidden dimension")
    if validate:
        _check_types("node_types", node_types, node_table.shape[0])
        _check_types("edge_types", edge_types, edge_table.shape[0])
    _require_i64("src", src)
    V, kv = node_types.shape
    E, ke = edge_types.shape
    h = node_table.shape[1]
    if src.numel() != E:
        raise ValueError("src must have one entry per edge")
    if records is not None and (records.dtype != torch.int32 or records.shape != (E, 4) or not records.is_contiguous()):
        raise ValueError("records must be the (E, 4) int32 embed_edge_records of this graph")
    ld = h if pitch is None else int(pitch)  # row-padded H0 / S views (as dmpnn_init's pitch)
    H0 = padded_rows(E, h, ld, node_table.dtype, dev)
    S = None if seg_ptr is None else padded_rows(V, h, ld, node_table.dtype, dev)
    _run(dev, _lib.load().nt_dmpnn_init_embed,
         _ptr(node_table), node_table.shape[0], _ptr(node_types), kv, _ptr(edge_table),
         edge_table.shape[0], _ptr(edge_types), ke, _ptr(src), _ptr(seg_ptr), _ptr(perm), V, E, h,
         act[0], act[1], reduce_code(reduce), code, _ptr(H0), _ptr(S), _ptr(amax), 0 if ld == h else ld,
         _ptr(records), _stream(dev))
    return H0, S


def embed_edge_records(node_types: Tensor, num_node_types: int, edge_types: Tensor, num_edge_types: int,
                       src: Tensor, perm: Tensor) -> Tensor:
    """(E, 4) int32 type records of a graph for dmpnn_init_embed (nt_embed_edge_records): per position of
    the dst CSR permutation, the in-edge and its 7 node-type and 2 edge-type indices as bytes (255 =
    out of range).  Build once per graph."""
    dev = _require_device(node_types, edge_types, src, perm)
    _require_i64("node_types", node_types)
    _require_i64("edge_types", edge_types)
    _require_i64("src", src)
    if node_types.dim() != 2 or node_types.shape[1] != 7 or edge_types.dim() != 2 or edge_types.shape[1] != 2:
        raise ValueError("type records need 7 node-type and 2 edge-type columns")
    V, E = node_types.shape[0], edge_types.shape[0]
    if perm.dtype != torch.int32 or perm.numel() != E or src.numel() != E:
        raise ValueError("perm (int32) and src need one entry per edge")
    out = torch.empty(max(E, 1), 4, dtype=torch.int32, device=dev)[:E]
    _run(dev, _lib.load().nt_embed_edge_records, _ptr(node_types.contiguous()), int(num_node_types),
         _ptr(edge_types.contiguous()), int(num_edge_types), _ptr(src), _ptr(perm), V, E, _ptr(out), _stream(dev))
    return out


# ------------------------------------------------------------------------------------ attention readouts
def node_scores(X: Tensor, *, a: Tensor | None = None, a_bias: Tensor | None = None,
                Q: Tensor | None = None, node_seg: Tensor | None = None,
                sqrt_key: float = 1.0) -> Tensor:
    """Per-node readout scores (fp32): X @ a + a_bias (Gated) or (Q[node_seg] * X).sum(1) / sqrt_key
    (SDPAttention)."""
    dev = _require_device(X, a, a_bias, Q, node_seg)
    code = _require_feat("X", X)
    n, h = X.shape
    if (a is None) == (Q is None):
        raise ValueError("pass exactly one of a (Gated) and Q (SDPAttention)")
    if a is not None:
        _require_feat("a", a, X.dtype)
        if a.numel() != h:
            raise ValueError("a must have h entries")
        if a_bias is not None:
            _require_feat("a_bias", a_bias, X.dtype)
    else:
        _require_feat("Q", Q, X.dtype)
        if Q.dim() != 2 or Q.shape[1] != h:
            raise RuntimeError(f"Q must be b x {h}, got {tuple(Q.shape)}")
        if node_seg is None:
            raise ValueError("SDPAttention scores need batch_node_index")
        _require_i64("batch_node_index", node_seg)
    s = torch.empty(n, dtype=torch.float32, device=dev)
    _run(dev, _lib.load().nt_node_scores,
         _ptr(X), n, h, _ptr(a), _ptr(a_bias), _ptr(Q), _ptr(node_seg), float(sqrt_key), code,
         _ptr(s), _stream(dev))
    return s


def softmax_pool(X: Tensor, scores: Tensor, seg_ptr: Tensor, perm: Tensor | None, nseg: int) -> Tensor:
    """out[g] = sum over v in segment g of softmax_g(scores)[v] * X[v]."""
    dev = _require_device(X, scores, seg_ptr, perm)
    code = _require_feat("X", X)
    if scores.dtype != torch.float32 or scores.numel() != X.shape[0]:
        raise ValueError("scores must be fp32 with one entry per row of X")
    if seg_ptr.dtype != torch.int32 or seg_ptr.numel() != nseg + 1:
        raise ValueError("seg_ptr must be int32 of length nseg + 1")
    h = X.shape[1]
    out = torch.empty(nseg, h, dtype=X.dtype, device=dev)
    _run(dev, _lib.load().nt_softmax_pool,
         _ptr(X), _ptr(scores), _ptr(seg_ptr), _ptr(perm), nseg, h, code, _ptr(out), _stream(dev))
    return out


def softmax_pool_backward(X: Tensor, scores: Tensor, seg_ptr: Tensor, perm: Tensor | None, node_seg: Tensor,
                          nseg: int, out: Tensor, dout: Tensor, *, a: Tensor | None = None,
                          Q: Tensor | None = None, sqrt_key: float = 1.0) -> tuple[Tensor, Tensor, Tensor]:
    """Backward of node_scores + softmax_pool for dout (nseg x h): (dX, ds, P) with ds the fp32 score
    gradient and P[g] = sum_{v in g} ds[v] X[v] (fp32): Gated da = P.sum(0), db = ds.sum(); SDPA
    dQ = P / sqrt_key (nt_softmax_pool_backward)."""
    dev = _require_device(X, scores, seg_ptr, perm, node_seg, out, dout, a, Q)
    code = _require_feat("X", X)
    _require_feat("out", out, X.dtype)
    _require_feat("dout", dout, X.dtype)
    if (a is None) == (Q is None):
        raise ValueError("pass exactly one of a (Gated) and Q (SDPAttention)")
    _require_feat("a" if a is not None else "Q", a if a is not None else Q, X.dtype)
    _require_i64("batch_node_index", node_seg)
    if scores.dtype != torch.float32 or scores.numel() != X.shape[0]:
        raise ValueError("scores must be fp32 with one entry per row of X")
    n, h = X.shape
    dX = torch.empty_like(X)
    ds = torch.empty(n, dtype=torch.float32, device=dev)
    P = torch.empty(nseg, h, dtype=torch.float32, device=dev)
    stats = torch.empty(max(3 * nseg, 1), dtype=torch.float32, device=dev)
    _run(dev, _lib.load().nt_softmax_pool_backward,
         _ptr(X), _ptr(scores), _ptr(seg_ptr), _ptr(perm), _ptr(node_seg), nseg, n, h, _ptr(out), _ptr(dout),
         _ptr(a), _ptr(Q), float(sqrt_key), code, _ptr(stats), _ptr(dX), _ptr(ds), _ptr(P), _stream(dev))
    return dX, ds, P


# ------------------------------------------------------------------------------------ dropout
def dropout_residual(Y: Tensor, p: float, seed: int, offset: int = 0, *, base: Tensor | None = None,
                     out: Tensor | None = None) -> Tensor:
    """out = (base or 0) + keep * Y / (1 - p), keep a counter-based hash of (seed, offset + i)
    (chemprop.py:26 Dropout + residual.py:28; see include/notorch_amd.h).  The same call on a
    gradient with base=None is the backward."""
    dev = _require_device(Y, base, out)
    code = _require_feat("Y", Y)
    if not Y.is_contiguous():
        raise ValueError("Y must be contiguous")
    if base is not None:
        _require_feat("base", base, Y.dtype)
        if base.shape != Y.shape or not base.is_contiguous():
            raise ValueError("base must be a contiguous tensor shaped like Y")
    if out is None:
        out = torch.empty_like(Y)
    else:
        _require_feat("out", out, Y.dtype)
        if out.shape != Y.shape or not out.is_contiguous():
            raise ValueError("out must be a contiguous tensor shaped like Y")
    _run(dev, _lib.load().nt_dropout_residual,
         _ptr(base), _ptr(Y), Y.numel(), float(p), int(seed) & (2**64 - 1), int(offset), code, _ptr(out),
         _stream(dev))
    return out


