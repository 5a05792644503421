"""Host-feed sweep on one GPU: bench.py's pipelined leg (DataLoader workers -> pinned -> side-stream
H2D overlapped with EmbeddedChempropBlock + Sum) at several worker counts, plus a cProfile of the
main process over one steady-state run.  Usage: python tools/feed_bench.py [--workers 8,14]"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workers", default="8,14")
    p.add_argument("--profile", action="store_true")
    a = p.parse_args()
    sys.argv = [sys.argv[0], "--steps", "20", "--warmup", "5", "--no-cpu-baseline"]
    import torch

    import bench

    args = bench.parse()
    env = bench.dist_env()
    dev = torch.device("cuda", 0)
    from notorch_amd import _lib

    _lib.load()
    res = bench.run_workload(args.workload, args, env, dev, headline=True)
    for w in [int(x) for x in a.workers.split(",")]:
        r = bench.pipeline_leg(res, dev, workers=w)
        print(json.dumps({k: r[k] for k in ("workers", "ms_per_batch", "device_step_ms", "ratio_to_device_step")}),
              flush=True)
    if a.profile:
        pr = cProfile.Profile()
        pr.enable()
        r = bench.pipeline_leg(res, dev, workers=int(a.workers.split(",")[-1]))
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
        print("profiled run", json.dumps({k: r[k] for k in ("workers", "ms_per_batch")}))
        print(s.getvalue())


if __name__ == "__main__":
    main()
