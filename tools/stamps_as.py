"""Per-phase cycles of the as16 update kernel from its diagnostic build (NT_AS_DIAG=1).
Usage: python tools/stamps_as.py [mols]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from notorch_amd import _lib, kernels as K  # noqa: E402
from notorch_amd.data.synth import make_batch  # noqa: E402

mols = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
lib = _lib.load()
fn = lib.nt_debug_as_stamps
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
G = make_batch("qm9", mols, seed=0).collate("nodes").to("cuda")
V, E, h = G.num_nodes, G.num_edges, 300
H = torch.randn(E, h, device="cuda"); S = torch.randn(V, h, device="cuda")
W = torch.randn(h, h, device="cuda") / 17; b = torch.randn(h, device="cuda")
Wp = K.pack_weights(W); src = G.edge_index[0].contiguous(); rev = G.rev_index
relu = K.act_code(torch.nn.ReLU())
os.environ["NT_UPDATE_KERNEL"] = "as"
out = K.dmpnn_update(H, S, src, rev, Wp, b, act=relu)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 7)()
for diag in ("0", "1"):
    os.environ["NT_AS_DIAG"] = diag
    fn(buf, 1)
    ts = []
    for _ in range(5):
        a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a_.record(); K.dmpnn_update(H, S, src, rev, Wp, b, act=relu, out=out); b_.record()
        torch.cuda.synchronize(); ts.append(a_.elapsed_time(b_) * 1e3)
    fn(buf, 0)
    print(f"diag={diag} E={E} launch us: {sorted(ts)[2]:.1f}")
waves = buf[4] / 5
names = ["gather+barrier", "mfma loop", "staging+barriers", "stores"]
print(f"waves/launch={waves:.0f}  span/launch (cycles, last launch)={buf[6] - buf[5]}")
for i, n in enumerate(names):
    print(f"{n:18s} {buf[i] / buf[4]:9.0f} cycles/wave")
