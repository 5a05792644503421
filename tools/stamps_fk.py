"""Per-phase cycle sums of update_fk_kernel, the shipping fp32 layer kernel, at config 2 (diagnostic
build: NT_LIB=diag, NT_FK_ABL=256 = the 128-row fused relu/sum instance with s_memtime stamps; results
valid).  A phase's time includes the waits its first instructions absorb (the MFMA phase waits for its
W and A fragments, the split for its gathered rows, the barrier for the slowest wave)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from notorch_amd import _lib, kernels as K  # noqa: E402
from notorch_amd.data.synth import make_batch  # noqa: E402

assert _lib.DIAG, "run with NT_LIB=diag"
lib = _lib.load()
fn = lib.nt_debug_pk_stamps
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
G = make_batch("qm9", 4096, seed=0).collate("nodes").to("cuda")
lay = G._nt_layout
V, E, h = G.num_nodes, G.num_edges, 300
H = torch.randn(E, h, device="cuda")
S = torch.randn(V, h, device="cuda")
Wp = K.pack_weights(torch.randn(h, h, device="cuda") / 17)
b = torch.randn(h, device="cuda")
src, rev = G.edge_index[0].contiguous(), G.rev_index
relu = K.act_code(torch.nn.ReLU())
deg = int((lay.dst_ptr[1:] - lay.dst_ptr[:-1]).max())
plan = K.tile_plan(lay.dst_ptr, E, deg, rows=128, ncu=K.PLAN_NCU)
rt = K.dmpnn_row_table(lay.dst_perm, plan[2], src, rev, V)
amax = torch.zeros(2, device="cuda")
K.absmax(H, amax[0:1])
K.absmax(S, amax[1:2])
out, S2 = torch.empty_like(H), torch.empty_like(S)
names = ["resid scale + MFMA", "W issue", "split + gather issue", "barrier", "epilogue", "-", "whole loop"]
for abl in sys.argv[1:] or ["256"]:
    os.environ["NT_FK_ABL"] = abl
    buf = (ctypes.c_ulonglong * 9)()
    fn(buf, 1)  # reset
    reps = 5
    for _ in range(reps):
        K.dmpnn_update_fused(H, S, src, rev, Wp, b, act=relu, plan=plan, tile_rows=128, max_in_degree=deg,
                             perm=lay.dst_perm, agg_act=relu, amax_in=amax, row_table=rt, out=out, S_out=S2)
    torch.cuda.synchronize()
    fn(buf, 0)
    waves = max(buf[7], 1)
    print(f"NT_FK_ABL={abl}: {waves} waves over {reps} launches; cycles per wave per launch (s_memtime ticks):")
    for q, n in enumerate(names):
        print(f"  {n:18s} {buf[q] / waves:12.0f}")
# launch time of the stamped and the plain instance (s_memtime ticks per µs of the launch)
for abl in ("256", "0"):
    os.environ["NT_FK_ABL"] = abl
    ts = []
    for _ in range(10):
        a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a_.record()
        K.dmpnn_update_fused(H, S, src, rev, Wp, b, act=relu, plan=plan, tile_rows=128, max_in_degree=deg,
                             perm=lay.dst_perm, agg_act=relu, amax_in=amax, row_table=rt, out=out, S_out=S2)
        b_.record()
        b_.synchronize()
        ts.append(a_.elapsed_time(b_) * 1e3)
    print(f"NT_FK_ABL={abl}: launch {sorted(ts)[len(ts) // 2]:.1f} us (median of 10)")
