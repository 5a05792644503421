"""Timing of nt_segment_reduce on the config-2 shapes: the Sum readout (V node rows -> B molecules)
and the backward's dXv (E edge rows -> V nodes by the src CSR).  Usage: python tools/seg_bench.py"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from notorch_amd import kernels as K  # noqa: E402
from notorch_amd.data.synth import make_batch  # noqa: E402


def timeit(fn, reps=20):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


G = make_batch("qm9", 4096, seed=0).collate("nodes").to("cuda")
V, E, h, B = G.num_nodes, G.num_edges, 300, len(G)
X = torch.randn(V, h, device="cuda")
Y = torch.randn(E, h, device="cuda")
mol_ptr, mol_perm = K.csr_build(G.batch_node_index.contiguous(), B)
src_ptr, src_perm = K.csr_build(G.edge_index[0].contiguous(), V)
fns = {"readout": lambda: K.segment_reduce(X, mol_ptr, mol_perm, B, reduce="sum"),
       "dXv": lambda: K.segment_reduce(Y, src_ptr, src_perm, V, reduce="sum")}
for f in fns.values():
    f()
torch.cuda.synchronize()
for name, f in fns.items():
    t = statistics.median(timeit(f) for _ in range(3))
    print(f"{name}: {t:.1f} us")
