"""Molecule-sharded data parallelism: independent units, no data-path collective.

Molecules share no edges, so a batch splits into contiguous molecule ranges that each GPU
collates and runs on its own.  The only collectives are bench bookkeeping (a barrier and two
scalar all-reduces for max-time / total-units), never on the forward path.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np


def edge_balanced_ranges(edges_per_mol: np.ndarray, world_size: int) -> list[tuple[int, int]]:
    """Contiguous [start, stop) molecule ranges, cut where the edge prefix sum crosses
    k * E_total / world_size (edge-balanced; matters for skewed polymer batches)."""
    e = np.asarray(edges_per_mol, dtype=np.int64)
    B = len(e)
    if world_size < 1:
        raise ValueError("world_size must be >= 1")
    if B == 0:
        return [(0, 0)] * world_size
    csum = np.cumsum(e)
    total = int(csum[-1])
    cuts = [0]
    for k in range(1, world_size):
        target = k * total / world_size
        i = int(np.searchsorted(csum, target, side="left"))  # first prefix reaching the target
        # cut before or after the molecule that crosses the target, whichever lands closer
        before = csum[i - 1] if i > 0 else 0
        after = csum[i] if i < B else total
        c = i if (target - before) <= (after - target) else i + 1
        c = min(max(c, cuts[-1]), B)
        cuts.append(c)
    cuts.append(B)
    return [(cuts[i], cuts[i + 1]) for i in range(world_size)]


@dataclass
class DistEnv:
    rank: int
    world_size: int
    local_rank: int

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


def dist_env() -> DistEnv:
    return DistEnv(
        int(os.environ.get("RANK", 0)),
        int(os.environ.get("WORLD_SIZE", 1)),
        int(os.environ.get("LOCAL_RANK", 0)),
    )


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_local_ranks(argv: list[str], nprocs: int, master_port: int | None = None,
                       poll_s: float = 0.2) -> int:
    """Start ``nprocs`` rank processes of ``[sys.executable, *argv]`` on this node, the way
    ``torch.distributed.run --nnodes 1 --nproc-per-node nprocs --master-addr 127.0.0.1`` would
    (RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT in each child's
    environment), and wait for them.  Children inherit stdout / stderr, so rank 0's output is
    relayed as it is written.  Returns 0 when every rank exits 0; otherwise the first failing
    rank's exit status (a signal -> 128 + signo), after terminating the ranks still running (by
    their own PIDs).  The caller must not have touched the GPU: the children are new processes
    (never an exec of the caller)."""
    import signal
    import subprocess
    import sys
    import time

    if nprocs < 1:
        raise ValueError("nprocs must be >= 1")
    port = master_port or _free_port()
    procs = []
    for r in range(nprocs):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs),
                   LOCAL_WORLD_SIZE=str(nprocs), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, *argv], env=env))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    for q in live:
                        q.send_signal(signal.SIGTERM)
            if live:
                time.sleep(poll_s)
    finally:
        # normal exit: nothing is left running.  On an exception / KeyboardInterrupt in the parent,
        # signal every rank still running first, then wait on one shared deadline, then kill.
        running = [p for p in procs if p.poll() is None]
        for p in running:
            try:
                p.send_signal(signal.SIGTERM)
            except ProcessLookupError:
                pass
        deadline = time.monotonic() + 30.0
        for p in running:
            try:
                p.wait(timeout=max(0.0, deadline - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc


def aggregate_throughput(local_units: float, local_seconds: float, device=None) -> tuple[float, float, float]:
    """(total_units, max_seconds, aggregate_rate) over all ranks; identity when not distributed.

    Uses two scalar all-reduces (SUM of units, MAX of time) on the default process group.
    """
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return local_units, local_seconds, local_units / local_seconds
    t = torch.tensor([local_units], dtype=torch.float64, device=device)
    s = torch.tensor([local_seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    dist.all_reduce(s, op=dist.ReduceOp.MAX)
    units, secs = float(t.item()), float(s.item())
    return units, secs, units / secs
