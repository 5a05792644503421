"""Per-role wait/busy cycles of the pk ring kernel (diagnostic build NT_PK_DIAG=1)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from notorch_amd import _lib, kernels as K  # noqa: E402
from notorch_amd.data.synth import make_batch  # noqa: E402

mols = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
lib = _lib.load()
fn = lib.nt_debug_pk_stamps
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
G = make_batch("qm9", mols, seed=0).collate("nodes").to("cuda")
lay = G._nt_layout
V, E, h = G.num_nodes, G.num_edges, 300
H = torch.randn(E, h, device="cuda"); S = torch.randn(V, h, device="cuda")
W = torch.randn(h, h, device="cuda") / 17; b = torch.randn(h, device="cuda")
Wp = K.pack_weights(W); src = G.edge_index[0].contiguous(); rev = G.rev_index
relu = K.act_code(torch.nn.ReLU())
deg = int((lay.dst_ptr[1:] - lay.dst_ptr[:-1]).max())
plan = K.tile_plan(lay.dst_ptr, E, deg)
out = torch.empty_like(H); S2 = torch.empty_like(S)
names = ["C ready waits", "C stage_free waits", "C whole", "P freed waits", "P stage_ready waits",
         "P finish", "P whole"]
os.environ["NT_FUSED_KERNEL"] = "pk"
for mode in ("fused", "unfused"):
    buf = (ctypes.c_ulonglong * 9)()
    for diag in ("0", "1"):
        os.environ["NT_PK_DIAG"] = diag
        fn(buf, 1)
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            K.dmpnn_update_fused(H, S, src, rev, Wp, b, act=relu,
                                 plan=plan if mode == "fused" else None, perm=lay.dst_perm,
                                 agg_act=relu, out=out, S_out=S2 if mode == "fused" else None)
            e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1) * 1e3)
        fn(buf, 0)
        print(f"{mode} diag={diag} launch us: {sorted(ts)[2]:.1f}")
    cw, pw = max(buf[7], 1), max(buf[8], 1)
    for i, n in enumerate(names):
        print(f"  {n:20s} {buf[i] / (cw if i < 3 else pw) / 5:10.0f} ticks/wave/launch")
