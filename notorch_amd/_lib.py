"""ctypes binding of the C-ABI library ``notorch_amd/lib/libnotorch_amd.so``.

The library is the only compute path of this package: there is no CPU or eager-torch fallback for
the forward kernels.  If the shared object is missing, every op raises :class:`NativeLibraryError`
(build it with ``python -c "import __graft_entry__ as g; g.build()"`` or ``make``).

Signatures mirror ``include/notorch_amd.h`` one-to-one.
"""
from __future__ import annotations

import ctypes
import os
import threading

_LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
# NT_LIB=diag loads the diagnostic build (make DIAG=1: A/B kernel variants selectable by NT_*
# environment variables, ablation / stamp builds); the default is the shipping library.
# NT_LIB=variant:<name> loads lib/libnotorch_amd_<name>.so, an A/B build of the shipping sources
# (make VARIANT=<name> EXTRA=-D...; tools only).
_NT_LIB = os.environ.get("NT_LIB", "")
DIAG = _NT_LIB == "diag"
if _NT_LIB.startswith("variant:"):
    LIB_PATH = os.path.join(_LIB_DIR, f"libnotorch_amd_{_NT_LIB.split(':', 1)[1]}.so")
else:
    LIB_PATH = os.path.join(_LIB_DIR, "libnotorch_amd_diag.so" if DIAG else "libnotorch_amd.so")
ABI_VERSION = 8

NT_F32, NT_BF16 = 0, 1
NT_SUM, NT_MEAN, NT_MAX, NT_MIN = 0, 1, 2, 3
REDUCE_CODES = {"sum": NT_SUM, "mean": NT_MEAN, "max": NT_MAX, "min": NT_MIN}
(
    NT_ACT_IDENTITY,
    NT_ACT_RELU,
    NT_ACT_LEAKY_RELU,
    NT_ACT_ELU,
    NT_ACT_GELU,
    NT_ACT_SILU,
    NT_ACT_TANH,
    NT_ACT_SIGMOID,
) = range(8)

_c_int, _c_i64, _c_f32, _c_size, _vp = (
    ctypes.c_int,
    ctypes.c_int64,
    ctypes.c_float,
    ctypes.c_size_t,
    ctypes.c_void_p,
)

# name -> (restype, argtypes); kept in header order (tests check this table against the header)
SIGNATURES: dict[str, tuple] = {
    "nt_abi_version": (_c_int, []),
    "nt_last_error": (ctypes.c_char_p, []),
    "nt_last_kernel": (ctypes.c_char_p, []),
    "nt_embed_bag": (_c_int, [_vp, _c_i64, _vp, _c_i64, _c_i64, _c_i64, _c_int, _vp, _vp]),
    "nt_dmpnn_init_embed": (
        _c_int,
        [_vp, _c_i64, _vp, _c_i64, _vp, _c_i64, _vp, _c_i64, _vp, _vp, _vp, _c_i64, _c_i64, _c_i64,
         _c_int, _c_f32, _c_int, _c_int, _vp, _vp, _vp, _c_i64, _vp, _vp],
    ),
    "nt_embed_edge_records": (_c_int, [_vp, _c_i64, _vp, _c_i64, _vp, _vp, _c_i64, _c_i64, _vp, _vp]),
    "nt_collate_graphs": (
        _c_int,
        [_c_i64, _vp, _vp, _c_i64, _vp, _vp, _c_i64, _vp, _vp, _c_int, _vp, _vp, _vp, _vp, _vp, _vp,
         _vp, _vp, _vp],
    ),
    "nt_csr_workspace_bytes": (_c_size, [_c_i64, _c_i64]),
    "nt_csr_build": (_c_int, [_vp, _c_i64, _c_i64, _vp, _vp, _vp, _c_size, _vp, _vp]),
    "nt_dmpnn_init": (
        _c_int,
        [_vp, _vp, _vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _c_int, _c_f32, _c_int, _c_int, _vp, _vp, _vp, _c_i64,
         _c_int, _vp],
    ),
    "nt_absmax": (_c_int, [_vp, _c_i64, _c_int, _vp, _vp]),
    "nt_segment_reduce": (
        _c_int,
        [_vp, _vp, _vp, _c_i64, _c_i64, _c_int, _c_int, _c_f32, _c_int, _vp, _vp],
    ),
    "nt_dmpnn_aggregate": (_c_int, [_vp, _vp, _vp, _c_i64, _c_i64, _c_int, _c_int, _vp, _vp]),
    "nt_segment_reduce_chunked": (
        _c_int,
        [_vp, _vp, _vp, _c_i64, _vp, _vp, _vp, _c_i64, _vp, _c_i64, _c_i64, _c_int, _c_int, _c_f32, _c_int, _vp, _vp,
         _vp, _vp],
    ),
    "nt_dmpnn_init_chunked": (
        _c_int,
        [_vp, _vp, _vp, _vp, _vp, _c_i64, _vp, _vp, _vp, _c_i64, _vp, _c_i64, _c_i64, _c_i64, _c_int, _c_f32, _c_int,
         _c_int, _vp, _vp, _vp, _vp, _c_i64, _vp, _c_i64, _vp],
    ),
    "nt_dmpnn_packed_weight_bytes": (_c_size, [_c_i64, _c_int]),
    "nt_dmpnn_pack_weight": (_c_int, [_vp, _c_i64, _c_i64, _c_int, _vp, _vp]),
    "nt_dmpnn_pack_weight_fk": (_c_int, [_vp, _c_i64, _c_i64, _vp, _vp]),
    "nt_dmpnn_pack_weights_fk": (_c_int, [_vp, _c_i64, _c_i64, _vp, _vp, _vp]),
    "nt_dmpnn_update": (
        _c_int,
        [_vp, _vp, _vp, _vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _c_int, _c_int, _c_f32, _c_int, _vp, _vp, _vp],
    ),
    "nt_dmpnn_tile_stride": (_c_i64, [_c_i64, _c_int, _c_int, _c_int]),
    "nt_dmpnn_tile_count": (_c_i64, [_c_i64, _c_i64]),
    "nt_dmpnn_tile_plan": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _c_i64, _vp, _vp]),
    "nt_dmpnn_tile_plan_hubs": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _c_int, _vp, _c_i64, _vp, _vp]),
    "nt_dmpnn_mark_hub_rows": (_c_int, [_vp, _c_i64, _vp, _c_i64, _c_int, _vp]),
    "nt_dmpnn_hub_aggregate": (
        _c_int, [_vp, _vp, _vp, _vp, _c_i64, _c_i64, _c_int, _c_int, _c_f32, _c_int, _vp, _vp, _c_i64, _vp],
    ),
    "nt_dmpnn_fused_tile_rows": (_c_int, [_c_i64, _c_int, _c_int, _c_int, _c_int]),
    "nt_dmpnn_update_fused": (
        _c_int,
        [_vp, _vp, _vp, _vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _c_int, _c_int, _c_f32, _vp, _c_i64,
         _c_int, _c_int, _vp, _vp, _vp, _c_int, _c_int, _c_f32, _c_int, _vp, _vp, _vp, _vp, _vp, _c_i64,
         _c_i64, _vp],
    ),
    "nt_dmpnn_hub_combine": (
        _c_int, [_vp, _vp, _vp, _c_i64, _vp, _c_i64, _c_i64, _c_int, _c_int, _vp, _vp, _c_i64, _vp],
    ),
    "nt_dmpnn_row_table": (_c_int, [_vp, _vp, _vp, _vp, _c_i64, _c_i64, _vp, _vp]),
    "nt_node_scores": (
        _c_int, [_vp, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _c_f32, _c_int, _vp, _vp],
    ),
    "nt_softmax_pool": (_c_int, [_vp, _vp, _vp, _vp, _c_i64, _c_i64, _c_int, _vp, _vp]),
    "nt_softmax_pool_backward": (_c_int, [_vp, _vp, _vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp,
                                          _c_f32, _c_int, _vp, _vp, _vp, _vp, _vp]),
    "nt_dmpnn_message": (
        _c_int,
        [_vp, _vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _c_int, _c_f32, _c_int, _vp, _vp],
    ),
    "nt_dmpnn_edge_backward": (
        _c_int,
        [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _c_int, _c_int, _c_f32,
         _c_int, _c_int, _vp, _vp, _vp],
    ),
    "nt_gather_rows": (_c_int, [_vp, _vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _c_int, _vp, _vp, _vp]),
    "nt_dropout_residual": (_c_int, [_vp, _vp, _c_i64, ctypes.c_float, ctypes.c_uint64, ctypes.c_uint64,
                                     _c_int, _vp, _vp]),
    "nt_segment_arg": (_c_int, [_vp, _vp, _vp, _c_i64, _c_i64, _c_int, _c_int, _c_f32, _c_int, _vp, _vp]),
    "nt_dmpnn_edge_backward_arg": (
        _c_int,
        [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _c_int, _c_int, _c_f32, _c_int, _vp,
         _vp, _vp],
    ),
    "nt_gather_rows_arg": (_c_int, [_vp, _vp, _vp, _vp, _c_i64, _c_i64, _c_int, _vp, _vp, _vp]),
    "nt_dmpnn_dense_matmul": (_c_int, [_vp, _c_i64, _c_i64, _vp, _c_int, _vp, _vp, _vp, _vp]),
    "nt_dmpnn_weight_grad_workspace": (_c_i64, [_c_i64, _c_i64]),
    "nt_dmpnn_weight_grad": (
        _c_int,
        [_vp, _vp, _vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _c_int, _c_f32, _c_int, _vp, _c_i64, _vp, _vp, _vp],
    ),
    "nt_dmpnn_weight_grad_fk": (
        _c_int,
        [_vp, _vp, _vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _c_int, _c_f32, _vp, _vp, _c_int, _vp, _c_i64, _vp, _vp,
         _vp],
    ),
}


class NativeLibraryError(RuntimeError):
    """The HIP extension is missing, stale or returned an error."""


_lock = threading.Lock()
_lib: ctypes.CDLL | None = None


def load() -> ctypes.CDLL:
    """Load (once) and type the C-ABI library.  Raises NativeLibraryError if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryError(
                f"notorch_amd HIP extension not built: {LIB_PATH} is missing "
                "(run `make` or __graft_entry__.build())"
            )
        # torch first: its bundled libamdhip64.so.7 then satisfies the library's DT_NEEDED, so the
        # kernels run on the same HIP runtime (and streams) as PyTorch.
        import torch  # noqa: F401

        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        ver = lib.nt_abi_version()
        if ver != ABI_VERSION:
            raise NativeLibraryError(f"libnotorch_amd ABI {ver} != expected {ABI_VERSION}; rebuild")
        _lib = lib
        return lib


def check(status: int) -> None:
    if status != 0:
        msg = load().nt_last_error().decode(errors="replace")
        raise NativeLibraryError(f"notorch_amd: {msg} (status {status})")
