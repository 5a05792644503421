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


def _pipeline_worker(rank, world, port, out):
    """One rank of a molecule-sharded forward: shard -> collate (fixed rev mode) -> .to(device) ->
    embedding + D-MPNN block + Sum readout (the oracle restatement stands in for the device kernels:
    there is no GPU here) -> readouts gathered to rank 0 (bookkeeping only, after the forward)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from notorch_amd.data.synth import make_batch
    from oracle import dmpnn_ref

    batch = make_batch("qm9", 48, seed=7)
    a, b = edge_balanced_ranges(2 * batch.n_bonds, world)[rank]
    G = batch.subset(a, b).collate("edges").to("cpu")
    torch.manual_seed(0)
    h = 32
    emb_v, emb_e = torch.nn.EmbeddingBag(42, h, mode="sum"), torch.nn.EmbeddingBag(13, h, mode="sum")
    blk_W = [torch.randn(h, h) / 6 for _ in range(3)]
    blk_b = [torch.randn(h) * 0.1 for _ in range(3)]
    with torch.no_grad():
        Xv, Xe = emb_v(G.node_feats), emb_e(G.edge_feats)
        node, _ = dmpnn_ref.chemprop_block(Xv, Xe, G.edge_index, G.rev_index, blk_W, blk_b)
        r = dmpnn_ref.readout(node, G.batch_node_index, len(G), "sum")
    sizes = [None] * world
    dist.all_gather_object(sizes, (a, b, G.num_nodes, G.num_edges))
    parts = [torch.zeros(sb - sa, h) for sa, sb, _, _ in sizes]
    dist.all_gather(parts, r)
    if rank == 0:
        out["parts"] = torch.cat(parts).numpy()
        out["sizes"] = sizes
    dist.destroy_process_group()


def test_gloo_world2_sharded_forward_pipeline():
    """The N>1 path end to end on CPU (gloo, world 2): every rank runs its edge-balanced shard's
    forward independently; the gathered readouts equal the whole batch's forward (fixed rev mode:
    molecules are independent units), and the shards' collated sizes add up."""
    from notorch_amd.data.synth import make_batch
    from oracle import dmpnn_ref

    mgr = mp.Manager()
    out = mgr.dict()
    port = 29600 + os.getpid() % 1000
    mp.spawn(_pipeline_worker, args=(2, port, out), nprocs=2, join=True)
    batch = make_batch("qm9", 48, seed=7)
    G = batch.collate("edges")
    torch.manual_seed(0)
    h = 32
    emb_v, emb_e = torch.nn.EmbeddingBag(42, h, mode="sum"), torch.nn.EmbeddingBag(13, h, mode="sum")
    blk_W = [torch.randn(h, h) / 6 for _ in range(3)]
    blk_b = [torch.randn(h) * 0.1 for _ in range(3)]
    with torch.no_grad():
        Xv, Xe = emb_v(G.node_feats), emb_e(G.edge_feats)
        node, _ = dmpnn_ref.chemprop_block(Xv, Xe, G.edge_index, G.rev_index, blk_W, blk_b)
        ref = dmpnn_ref.readout(node, G.batch_node_index, len(G), "sum").numpy()
    sizes = out["sizes"]
    assert sizes[0][0] == 0 and sizes[0][1] == sizes[1][0] and sizes[1][1] == 48
    assert sizes[0][2] + sizes[1][2] == G.num_nodes and sizes[0][3] + sizes[1][3] == G.num_edges
    np.testing.assert_allclose(out["parts"], ref, rtol=1e-5, atol=1e-5)


def test_bench_gpus_n_launches_its_own_ranks():
    """`python bench.py --gpus 2` with no external launcher starts 2 rank processes itself (before
    any GPU call) and relays rank 0's line: n_gpus = 2, units summed and time maxed over ranks."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["units"] == 3000.0 and d["max_seconds"] == 2.0


def test_bench_rejects_world_size_mismatch():
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def test_launcher_propagates_a_failing_rank(tmp_path):
    """One rank exiting non-zero makes launch_local_ranks return non-zero and stop the others."""
    import time

    from notorch_amd.shard import launch_local_ranks

    script = tmp_path / "w.py"
    script.write_text("import os, sys, time\n"
                      "r = int(os.environ['RANK'])\n"
                      "assert os.environ['WORLD_SIZE'] == '3' and os.environ['MASTER_ADDR'] == '127.0.0.1'\n"
                      "sys.exit(7) if r == 1 else time.sleep(120)\n")
    t0 = time.time()
    rc = launch_local_ranks([str(script)], 3)
    assert rc == 7 and time.time() - t0 < 60
