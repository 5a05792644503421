"""Host enqueue cost of one config-2 step (ChempropBlock + Sum) against its device time, eager and as
a hipGraph replay (notorch_amd.graphs.GraphedForward), for short timed regions like the driver's
(--steps 20).  Usage: python tools/cpu_overhead.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from notorch_amd.data.synth import make_batch  # noqa: E402
from notorch_amd.graphs import GraphedForward  # noqa: E402
from notorch_amd.nn import ChempropBlock, Sum  # noqa: E402

dev = torch.device("cuda")
G = make_batch("qm9", 4096, seed=1000).collate("nodes")
torch.manual_seed(0)
h = 300
G = G.update(node_feats=torch.randn(G.num_nodes, h), edge_feats=torch.randn(G.num_edges, h)).to(dev)
blk, ro = ChempropBlock(hidden_dim=h, depth=3).to(dev).eval(), Sum()
step = lambda: ro(blk(G))  # noqa: E731
with torch.no_grad():
    for _ in range(200):
        step()
    torch.cuda.synchronize()
    for n in (20, 50):
        t0 = time.perf_counter()
        for _ in range(n):
            step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"eager {n} steps: enqueue {(t1 - t0) / n * 1e6:.1f} us/step, total {(t2 - t0) / n * 1e6:.1f} us/step")
    fwd = GraphedForward(lambda g: ro(blk(g)), G)
    for _ in range(200):
        fwd()
    torch.cuda.synchronize()
    for n in (20, 50):
        t0 = time.perf_counter()
        for _ in range(n):
            fwd()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"graph {n} steps: enqueue {(t1 - t0) / n * 1e6:.1f} us/step, total {(t2 - t0) / n * 1e6:.1f} us/step")
