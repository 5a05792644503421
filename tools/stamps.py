"""Per-phase cycle shares of the x6 update K-step from the diagnostic stamp build."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from notorch_amd import _lib, kernels as K  # noqa: E402
from notorch_amd.data.synth import make_batch  # noqa: E402

mols = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
lib = _lib.load()
fn = lib.nt_debug_x6_stamps
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
G = make_batch("qm9", mols, seed=0).collate("nodes").to("cuda")
V, E, h = G.num_nodes, G.num_edges, 300
H = torch.randn(E, h, device="cuda"); S = torch.randn(V, h, device="cuda")
W = torch.randn(h, h, device="cuda") / 17; b = torch.randn(h, device="cuda")
Wp = K.pack_weights(W); src = G.edge_index[0].contiguous(); rev = G.rev_index
os.environ["NT_UPDATE_KERNEL"] = "x6"
os.environ["NT_X6_CFG"] = "s"
relu = K.act_code(torch.nn.ReLU())
out = K.dmpnn_update(H, S, src, rev, Wp, b, act=relu)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 5)()
fn(buf, 1)
for _ in range(5):
    K.dmpnn_update(H, S, src, rev, Wp, b, act=relu, out=out)
torch.cuda.synchronize()
fn(buf, 1)
names = ["dma_issue", "a_read_split", "mfma+b_reads", "barrier_wait"]
tot = sum(buf[i] for i in range(4))
steps = buf[4]
print(f"E={E} wave-steps={steps}")
for i, n in enumerate(names):
    print(f"{n:14s} {buf[i] / tot * 100:5.1f} %   {buf[i] / steps:8.0f} cycles/step")
