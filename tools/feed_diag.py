"""Where the pipelined host feed's time goes (one GPU): (a) the DataLoader + pin + H2D alone, no model;
(b) the model on fresh device batches copied from already-pinned host batches (no workers);
(c) the full pipeline with the time the main thread spends in next() vs enqueueing the forward.
Usage: python tools/feed_diag.py [--workers 8]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workers", type=int, default=8)
    p.add_argument("--pin-threads", type=int, default=0)
    p.add_argument("--ring-slots", type=int, default=3)
    p.add_argument("--profile", action="store_true")
    p.add_argument("--background", action="store_true", help="issue H2D on the prefetcher's own thread")
    a = p.parse_args()
    import torch

    from notorch_amd import _lib
    from notorch_amd.data.loader import GraphCollator, graph_loader
    from notorch_amd.data.models.graph import BatchedGraph
    from notorch_amd.data.synth import make_batch
    from notorch_amd.nn import ChempropBlock, EmbeddedChempropBlock, GraphEmbedding, Sum

    _lib.load()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    enc = EmbeddedChempropBlock(GraphEmbedding(42, 13, 300), ChempropBlock(hidden_dim=300, depth=3), fuse=True)
    enc = enc.to(dev).eval()
    readout = Sum()
    graphs = make_batch("qm9", 4096, seed=1000).to_graphs()
    W = a.workers
    warm, n = W * 3 + 4, 3 * W
    out = {"workers": W, "pin_threads": a.pin_threads, "ring_slots": a.ring_slots, "background": a.background}

    def run_loader(model: bool):
        loader = graph_loader(graphs * (warm + n), 4096, dev, num_workers=W, pin_threads=a.pin_threads,
                              ring_slots=a.ring_slots, background=a.background)
        it = iter(loader)
        with torch.no_grad():
            for _ in range(warm):
                G = next(it)
                if model:
                    readout(enc(G))
            torch.cuda.synchronize(dev)
            t_next = t_fwd = 0.0
            t0 = time.perf_counter()
            k = 0
            while True:
                t1 = time.perf_counter()
                try:
                    G = next(it)
                except StopIteration:
                    break
                t2 = time.perf_counter()
                if model:
                    readout(enc(G))
                t3 = time.perf_counter()
                t_next += t2 - t1
                t_fwd += t3 - t2
                k += 1
            torch.cuda.synchronize(dev)
            t = time.perf_counter() - t0
        if hasattr(loader.batches, "close"):
            loader.batches.close()
        del loader, it
        return {"ms_per_batch": t / k * 1e3, "next_ms": t_next / k * 1e3, "enqueue_ms": t_fwd / k * 1e3, "batches": k}

    # (a0) the workers alone: DataLoader without pinning or device copies
    dl = torch.utils.data.DataLoader(graphs * (warm + n), batch_size=4096, collate_fn=GraphCollator(),
                                     num_workers=W, persistent_workers=True, prefetch_factor=2)
    it = iter(dl)
    for _ in range(warm):
        next(it)
    t0 = time.perf_counter()
    k = sum(1 for _ in it)
    out["a0_workers_only"] = {"ms_per_batch": (time.perf_counter() - t0) / k * 1e3, "batches": k}
    del it, dl
    out["a_loader_only"] = run_loader(False)
    # (b) fresh batches from pinned host buffers, no workers
    coll = GraphCollator()
    hosts = [coll(graphs).pin_memory() for _ in range(4)]
    with torch.no_grad():
        for r in range(2):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            t_enq = 0.0
            for i in range(24):
                t1 = time.perf_counter()
                G = _copy_to(hosts[i % 4], dev)
                readout(enc(G))
                t_enq += time.perf_counter() - t1
            torch.cuda.synchronize(dev)
            t = time.perf_counter() - t0
        out["b_pinned_fresh"] = {"ms_per_batch": t / 24 * 1e3, "enqueue_ms": t_enq / 24 * 1e3}
        if a.profile:
            import cProfile
            import io
            import pstats

            pr = cProfile.Profile()
            pr.enable()
            for i in range(24):
                readout(enc(_copy_to(hosts[i % 4], dev)))
            pr.disable()
            torch.cuda.synchronize(dev)
            sio = io.StringIO()
            pstats.Stats(pr, stream=sio).sort_stats("tottime").print_stats(30)
            print(sio.getvalue(), flush=True)
        # resident: the same device batch again
        G = _copy_to(hosts[0], dev)
        for _ in range(5):
            readout(enc(G))
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(24):
            readout(enc(G))
        torch.cuda.synchronize(dev)
        out["b_resident"] = {"ms_per_batch": (time.perf_counter() - t0) / 24 * 1e3}
    out["c_pipeline"] = run_loader(True)
    print(json.dumps(out), flush=True)


def _copy_to(host, dev):
    import copy

    return copy.copy(host).to(dev, non_blocking=True)


if __name__ == "__main__":
    main()
