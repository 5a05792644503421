"""Step time of the config-2 forward with and without the bench's per-launch HIP events (the roofline
timer, _engine.UPDATE_EVENTS), interleaved rounds in one process: what the event records cost the
step.  Usage: python tools/event_cost.py [--workload qm9-4096] [--steps 50] [--rounds 5]"""
import argparse
import os
import statistics
import sys
import time
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from notorch_amd.nn import Sum  # noqa: E402
from notorch_amd.nn.gnn import _engine  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", default="qm9-4096")
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--rounds", type=int, default=5)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    kind, n_mols, h, depth, sdtype = bench.WORKLOADS[a.workload]
    embedding, block = bench.make_model(h, depth, sdtype == "bf16", dev)
    env = types.SimpleNamespace(rank=0, world_size=1, distributed=False)
    jobs, _, _ = bench.make_jobs(a.workload, 0, 1, dev, embedding)
    readout = Sum()

    def step():
        for j in jobs:
            readout(block(j.Gd))

    res = {"events": [], "no events": []}
    for _ in range(a.rounds):
        for mode in res:
            _engine.UPDATE_EVENTS = [] if mode == "events" else None
            t = bench.timed_steps(step, a.steps, 5, env, dev)
            res[mode].append(t / a.steps * 1e3)
    _engine.UPDATE_EVENTS = None
    for mode, v in res.items():
        print(f"{mode:10s} ms/step median {statistics.median(v):.4f} min {min(v):.4f}")


if __name__ == "__main__":
    main()
