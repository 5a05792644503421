"""Per-phase host time of one GraphFeeder batch (config 2: 4096 QM9-shaped molecules) on this
machine's CPU, single process, N repetitions: the C++ per-graph walk, the native collate + plans, the
pack into a slot and the skeleton pickle.  Usage: python tools/collate_phases.py [--reps 30]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=30)
    a = p.parse_args()
    import numpy as np
    import torch

    torch.set_num_threads(1)
    from notorch_amd.data.loader import SlotBatch, SlotRing
    from notorch_amd.data.models import graph as gm
    from notorch_amd.data.synth import make_batch

    Gs = make_batch("qm9", 4096, seed=1000).to_graphs()
    G0 = gm.BatchedGraph.from_graphs(Gs)
    ring = SlotRing(1, 1, G0.packed_nbytes() * 3 // 2)
    fast = gm._collate_py()
    t = {"graph_arrays": [], "collate_and_plans": [], "host_stats": [], "pack_into_slot": [], "skeleton_pickle": []}
    orig = gm.host_stats

    def timed_stats(*args, **kw):
        t0 = time.perf_counter()
        orig(*args, **kw)
        t["host_stats"].append(time.perf_counter() - t0)

    gm.host_stats = timed_stats
    for i in range(a.reps + 3):
        t0 = time.perf_counter()
        r = fast.graph_arrays(Gs)
        t1 = time.perf_counter()
        G = gm._native_collate(gm.BatchedGraph, Gs, "nodes", r, ring.slot(0))
        t2 = time.perf_counter()
        G.pack(out=ring.slot(0))
        t3 = time.perf_counter()
        SlotBatch.pack(G, ring, 0)
        t4 = time.perf_counter()
        if i >= 3:
            t["graph_arrays"].append(t1 - t0)
            t["collate_and_plans"].append(t2 - t1)
            t["pack_into_slot"].append(t3 - t2)
            t["skeleton_pickle"].append(t4 - t3 - (t3 - t2))  # SlotBatch.pack re-packs (no-op copies)
    t["host_stats"] = t["host_stats"][3:]
    print(json.dumps({k: round(float(np.median(v)) * 1e3, 3) for k, v in t.items()} | {"unit": "ms (median)"}))


if __name__ == "__main__":
    main()
