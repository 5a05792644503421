"""CPU: molecule sharding — edge-balanced contiguous ranges, and the N>1 bench
bookkeeping (max-time / total-units all-reduces) on a world_size-2 gloo group."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from notorch_amd.shard import aggregate_throughput, edge_balanced_ranges


def test_ranges_cover_and_balance():
    rng = np.random.default_rng(0)
    e = rng.integers(10, 30, size=1000)
    for n in (1, 2, 3, 8):
        rs = edge_balanced_ranges(e, n)
        assert rs[0][0] == 0 and rs[-1][1] == 1000
        assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
        loads = [e[a:b].sum() for a, b in rs]
        assert max(loads) - min(loads) <= 2 * e.max()


def test_ranges_skewed_polymer_like():
    e = np.array([1000, 10, 10, 10, 5000, 10, 10])
    rs = edge_balanced_ranges(e, 2)
    assert rs == [(0, 4), (4, 7)]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from notorch_amd.data.synth import make_batch

    batch = make_batch("qm9", 64, seed=7)
    rs = edge_balanced_ranges(2 * batch.n_bonds, world)
    a, b = rs[rank]
    shard = batch.subset(a, b)
    G = shard.collate("edges")
    units = G.num_edges * 3
    total, secs, rate = aggregate_throughput(units, 1.0 + rank)
    out[rank] = (a, b, G.num_edges, total, secs)
    dist.destroy_process_group()


def test_gloo_world2_sharding_and_aggregation():
    mgr = mp.Manager()
    out = mgr.dict()
    port = 29500 + os.getpid() % 1000
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    (a0, b0, e0, t0, s0), (a1, b1, e1, t1, s1) = out[0], out[1]
    assert a0 == 0 and b0 == a1 and b1 == 64
    assert t0 == t1 == 3 * (e0 + e1)      # SUM of units
    assert s0 == s1 == 2.0                # MAX of times
