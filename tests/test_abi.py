"""CPU: the C-ABI library loads and exports exactly what include/notorch_amd.h declares.
No compute call is made (no GPU here); only pure-host entry points are exercised."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "notorch_amd.h")


def header_functions():
    txt = open(HEADER).read()
    return re.findall(r"^NT_API\s+[\w\s\*]+?\b(nt_\w+)\s*\(", txt, flags=re.M)


def test_header_declares_the_boundary():
    names = header_functions()
    assert set(names) == {
        "nt_abi_version", "nt_last_error", "nt_last_kernel", "nt_csr_workspace_bytes", "nt_csr_build", "nt_dropout_residual",
        "nt_dmpnn_init", "nt_segment_reduce", "nt_dmpnn_aggregate", "nt_dmpnn_packed_weight_bytes",
        "nt_dmpnn_pack_weight", "nt_dmpnn_pack_weights_fk", "nt_dmpnn_update", "nt_dmpnn_tile_count", "nt_dmpnn_tile_plan",
        "nt_dmpnn_update_fused", "nt_dmpnn_message", "nt_dmpnn_edge_backward", "nt_gather_rows",
        "nt_embed_bag", "nt_dmpnn_init_embed", "nt_embed_edge_records", "nt_node_scores", "nt_softmax_pool",
        "nt_collate_graphs", "nt_segment_reduce_chunked",
        "nt_dmpnn_dense_matmul", "nt_dmpnn_weight_grad", "nt_dmpnn_weight_grad_workspace", "nt_segment_arg",
        "nt_dmpnn_edge_backward_arg", "nt_gather_rows_arg", "nt_absmax", "nt_dmpnn_fused_tile_rows",
        "nt_dmpnn_tile_stride", "nt_dmpnn_row_table", "nt_dmpnn_pack_weight_fk", "nt_dmpnn_tile_plan_hubs",
        "nt_dmpnn_mark_hub_rows", "nt_dmpnn_hub_aggregate", "nt_dmpnn_hub_combine", "nt_dmpnn_weight_grad_fk",
        "nt_softmax_pool_backward", "nt_dmpnn_init_chunked",
    }


def test_library_exports_every_header_symbol():
    from notorch_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail(f"{_lib.LIB_PATH} not built (run make)")
    lib = _lib.load()
    for name in header_functions():
        assert hasattr(lib, name), name
    # and the ctypes signature table covers exactly the header
    assert set(_lib.SIGNATURES) == set(header_functions())


def test_abi_version_and_errors_without_gpu():
    from notorch_amd import _lib

    lib = _lib.load()
    assert lib.nt_abi_version() == _lib.ABI_VERSION == 8
    assert lib.nt_last_kernel() == b""  # no layer call yet on this thread
    assert lib.nt_dmpnn_packed_weight_bytes(300, 0) > 0
    assert lib.nt_dmpnn_packed_weight_bytes(0, 0) == 0
    # argument validation happens before any device call: EINVAL + message
    rc = lib.nt_dmpnn_update(None, None, None, None, None, None, 0, 0, 0, 1, 1, 0.0, 0, None, None, None)
    assert rc == 1 and b"bad sizes" in lib.nt_last_error()
    # ABI 6: the fp32 split-scale workspace is the caller's (no library-owned device scratch); the
    # check precedes any device call, so fake aligned pointers reach it
    fake = [ctypes.c_void_p(0x1000 * (i + 1)) for i in range(6)]
    rc = lib.nt_dmpnn_update(*fake, 4, 8, 16, 1, 1, 0.0, 0, None, ctypes.c_void_p(0x9000), None)
    assert rc == 1 and b"amax_ws" in lib.nt_last_error()
    rc = lib.nt_dmpnn_dense_matmul(fake[0], 8, 16, fake[1], 0, None, None, fake[2], None)
    assert rc == 1 and b"amax_ws" in lib.nt_last_error()
    rc = lib.nt_segment_reduce(None, None, None, 4, 8, 9, 0, 0.0, 0, None, None)
    assert rc == 1 and b"reduce" in lib.nt_last_error()
    rc = lib.nt_segment_reduce(None, None, None, 4, 8, 0, 0, 0.0, 1, None, None)
    assert rc == 1 and b"NULL" in lib.nt_last_error()  # bf16 is implemented: validation reached
    rc = lib.nt_segment_reduce(None, None, None, 4, 8, 0, 0, 0.0, 7, None, None)
    assert rc == 3  # NT_EUNSUPPORTED: unknown dtype code
    rc = lib.nt_dmpnn_aggregate(None, None, None, 4, 8, 9, 0, None, None)  # = nt_segment_reduce, act relu
    assert rc == 1 and b"reduce" in lib.nt_last_error()
    rc = lib.nt_dmpnn_aggregate(None, None, None, 4, 8, 0, 0, None, None)
    assert rc == 1 and b"NULL" in lib.nt_last_error()
    assert lib.nt_dmpnn_packed_weight_bytes(512, 1) == 16 * 32 * 64 * 16  # bf16 image, h = 512
    rc = lib.nt_dmpnn_message(None, None, None, None, 4, 8, 16, 1, 0.0, 1, None, None)
    assert rc == 1 and b"NULL" in lib.nt_last_error()  # bf16 backward is implemented
    rc = lib.nt_dmpnn_message(None, None, None, None, 4, 8, 16, 1, 0.0, 7, None, None)
    assert rc == 3
    rc = lib.nt_csr_build(None, -1, 3, None, None, None, 0, None, None)
    assert rc == 1
    # backward entry points validate before touching the device
    rc = lib.nt_dmpnn_edge_backward(None, None, None, None, None, None, None, None, 4, 8, 16, 1, 1,
                                    0.0, 2, 0, None, None, None)
    # max / min aggregations take nt_dmpnn_edge_backward_arg; this entry point covers sum / mean
    assert rc == 3 and b"sum | mean" in lib.nt_last_error()
    rc = lib.nt_dmpnn_message(None, None, None, None, 4, 8, 16, 99, 0.0, 0, None, None)
    assert rc == 1
    rc = lib.nt_gather_rows(None, None, None, None, -1, 4, 8, 0, None, None, None)
    assert rc == 1


def test_abi7_row_pitch_and_hub_combine_checks_without_gpu():
    """ABI 7 arguments are validated before any device call: row pitches (fp32 only, >= h, % 4),
    hub partials (fp32 only), nt_dmpnn_hub_combine's sizes."""
    from notorch_amd import _lib

    lib = _lib.load()
    fake = [ctypes.c_void_p(0x1000 * (i + 1)) for i in range(12)]
    # nt_dmpnn_update_fused, bf16 with a padded input pitch: EUNSUPPORTED
    rc = lib.nt_dmpnn_update_fused(*fake[:6], 10, 20, 512, 1, 1, 0.0, None, 0, 64, 4, None, None, None, 0, 1, 0.0,
                                   1, None, None, fake[6], None, None, 520, 0, None)
    assert rc == 3 and b"fp32 only" in lib.nt_last_error()
    rc = lib.nt_dmpnn_update_fused(*fake[:6], 10, 20, 512, 1, 1, 0.0, None, 0, 64, 4, None, None, None, 0, 1, 0.0,
                                   1, None, None, fake[6], None, fake[7], 0, 0, None)
    assert rc == 3  # hub partials are fp32 only
    # nt_dmpnn_init: a padded pitch needs fp32
    rc = lib.nt_dmpnn_init(*fake[:5], 10, 20, 512, 1, 0.0, 0, 1, fake[5], fake[6], None, 520, 0, None)
    assert rc == 3 and b"ld_out" in lib.nt_last_error()
    # nt_dmpnn_init_chunked: pitch % 4
    rc = lib.nt_dmpnn_init_chunked(*fake[:5], 3, fake[5], None, None, 0, fake[6], 10, 20, 300, 1, 0.0, 0, 0,
                                   fake[7], fake[8], fake[9], None, 302, None, 0, None)
    assert rc == 1 and b"ld_out" in lib.nt_last_error()
    # nt_dmpnn_hub_combine: h % 4, pitch >= h
    rc = lib.nt_dmpnn_hub_combine(*fake[:3], 2, fake[3], 10, 6, 0, 0, None, fake[4], 0, None)
    assert rc == 1 and b"bad sizes" in lib.nt_last_error()
    rc = lib.nt_dmpnn_hub_combine(*fake[:3], 2, fake[3], 10, 8, 0, 0, None, fake[4], 4, None)
    assert rc == 1 and b"pitch" in lib.nt_last_error()
    rc = lib.nt_dmpnn_hub_combine(*fake[:3], 2, fake[3], 10, 8, 0, 1, None, fake[4], 0, None)
    assert rc == 3  # fp32 only


def test_check_raises_with_message():
    from notorch_amd import _lib

    lib = _lib.load()
    lib.nt_dmpnn_pack_weight(None, 1, 0, 0, None, None)
    with pytest.raises(_lib.NativeLibraryError, match="bad sizes"):
        _lib.check(1)


def test_weight_grad_host_checks():
    """nt_dmpnn_weight_grad's workspace query and argument validation (pure host, no launch)."""
    from notorch_amd import _lib

    lib = _lib.load()
    assert lib.nt_dmpnn_weight_grad_workspace(77_840, 300) > 0
    assert lib.nt_dmpnn_weight_grad_workspace(-1, 300) == -1
    rc = lib.nt_dmpnn_weight_grad(None, None, None, None, None, 4, 8, 16, 1, 0.0, 1, None, 0, None, None, None)
    assert rc == 3  # bf16 weight grad needs src / rev (the message is formed in the kernel): NULL here
    rc = lib.nt_dmpnn_weight_grad(None, None, None, None, None, 4, 8, 16, 1, 0.0, 0, None, 0, None, None, None)
    assert rc == 1 and b"dW_out" in lib.nt_last_error()
