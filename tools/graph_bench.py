"""Small-batch latency (32 QM9 molecules, h=300, d=3): eager forward vs the
hipGraph replay of the same forward (notorch_amd/graphs.py).  Usage: python tools/graph_bench.py [mols]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from notorch_amd.data.synth import make_batch  # noqa: E402
from notorch_amd.graphs import GraphedForward  # noqa: E402
from notorch_amd.nn import ChempropBlock, Sum  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
G = make_batch("qm9", n, seed=0).collate("nodes")
torch.manual_seed(0)
h = 300
Gd = G.update(node_feats=torch.randn(G.num_nodes, h), edge_feats=torch.randn(G.num_edges, h)).to("cuda")
blk, ro = ChempropBlock(h, depth=3).eval().cuda(), Sum()
fn = lambda G: ro(blk(G))  # noqa: E731
fwd = GraphedForward(fn, Gd)
E = G.num_edges
for name, call in (("eager", lambda: fn(Gd)), ("hipgraph", fwd)):
    with torch.no_grad():
        for _ in range(20):
            call()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        K = 500
        for _ in range(K):
            call()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / K
    print(f"{name:9s} {n} mols (E={E}): {dt * 1e6:8.1f} us/forward  {E * 3 / dt:.3e} edge-msg/s")
