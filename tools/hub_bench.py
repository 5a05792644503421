"""Device time of nt_dmpnn_hub_aggregate on the polymer-16 batch (config 5) for the library selected
by NT_LIB (A/B variant builds of csrc/hubs.hip).  Usage: python tools/hub_bench.py"""
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


G = make_batch("polymer", 16, seed=0).collate("nodes").to("cuda")
lay = G._nt_layout
V, E, h = G.num_nodes, G.num_edges, 300
deg = lay.dst_ptr[1:] - lay.dst_ptr[:-1]
hubs = torch.nonzero(deg > 32).flatten().to(torch.int32)
rows = int(deg[deg > 32].sum())
X = K.padded_rows(E, h, 304, torch.float32, "cuda")
X.copy_(torch.randn(E, h, device="cuda"))
out = K.padded_rows(V, h, 304, torch.float32, "cuda")
relu = K.act_code(torch.nn.ReLU())
f = lambda: K.hub_aggregate(X, lay.dst_perm, lay.dst_ptr, hubs, out, act=relu)  # noqa: E731
f()
torch.cuda.synchronize()
med = statistics.median(timeit(f) for _ in range(5))
print(f"hubs={hubs.numel()} hub rows={rows}: median {med:.1f} us  ({rows * h * 4 / (med * 1e-6) / 1e12:.2f} TB/s of rows)"
      f"  lib={os.environ.get('NT_LIB', '')}")
