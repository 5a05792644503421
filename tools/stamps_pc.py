"""Per-phase cycle shares of the producer/consumer update kernel (diagnostic stamp build)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from notorch_amd import _lib, kernels as K  # noqa: E402
from notorch_amd.data.synth import make_batch  # noqa: E402

mols = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
lib = _lib.load()
fn = lib.nt_debug_pc_stamps
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
G = make_batch("qm9", mols, seed=0).collate("nodes").to("cuda")
V, E, h = G.num_nodes, G.num_edges, 300
H = torch.randn(E, h, device="cuda"); S = torch.randn(V, h, device="cuda")
W = torch.randn(h, h, device="cuda") / 17; b = torch.randn(h, device="cuda")
Wp = K.pack_weights(W); src = G.edge_index[0].contiguous(); rev = G.rev_index
os.environ["NT_UPDATE_KERNEL"] = "pc"
os.environ["NT_PC_MODE"] = "1"
relu = K.act_code(torch.nn.ReLU())
out = K.dmpnn_update(H, S, src, rev, Wp, b, act=relu)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 9)()
fn(buf, 1)
for _ in range(5):
    K.dmpnn_update(H, S, src, rev, Wp, b, act=relu, out=out)
torch.cuda.synchronize()
fn(buf, 1)
cs, ps = max(buf[6], 1), max(buf[7], 1)
print(f"E={E} consumer wave-steps={buf[6]} producer wave-steps={buf[7]}")
print(f"consumer: compute {buf[0] / cs:7.0f}  barrier {buf[1] / cs:7.0f}  cycles/step")
print(f"producer: W-issue {buf[8] / ps:7.0f} (of total issue)")
print(f"producer: issue {buf[2] / ps:7.0f}  vmcnt-wait {buf[3] / ps:7.0f}  split {buf[4] / ps:7.0f}  barrier {buf[5] / ps:7.0f}  cycles/step")
