"""GraphFeeder: per-molecule Graph dataset -> collated batches in a page-locked slot ring, without
torch's DataLoader machinery (the host feed).

The reference feeds ``BatchedGraph.from_graphs`` (notorch/data/models/graph.py:186-223) from torch
DataLoader workers (notorch/data/dataset.py:56-71, transforms/graph.py:45).  With the collate itself
native (~3 ms per 4096 molecules on one core), what limits a DataLoader feed is the consumer
process's per-batch Python work: index lists out, results in, storage hand-offs.  Here:

* W worker processes are forked once (persistent) and own K slots each of a :class:`SlotRing`
  (shared memory mapped before the fork, page-locked in the parent after it).
* Each epoch the parent sends every worker its share of the batch order once (batch b goes to worker
  b mod W, into that worker's slot (b div W) mod K): no per-batch index traffic.
* A worker collates straight into the slot (``from_graphs(out=...)``), writes the batch's pickled
  skeleton (tensors as slot offsets) into the slot's tail and publishes the batch by storing its tag
  (epoch << 32 | b + 1) in the ring's flag word; the parent polls that word, rebuilds the batch as
  views of the slot and copies it to the device by DMA (``DevicePrefetcher``), then frees the slot.
* A batch that does not fit its slot travels through the worker's pipe instead (flag = -tag); a
  worker error travels the same way and is raised in the parent at that batch.
Workers run host code only (no HIP call); they are forked after the C-ABI library is loaded.
"""
from __future__ import annotations

import time
from typing import Optional, Sequence

import numpy as np
import torch

from notorch_amd.data.loader import SlotBatch, SlotRing
from notorch_amd.data.models.graph import BatchedGraph, Graph, RevOffset

META_BYTES = 1 << 16  # tail of every slot: 8-byte length + the batch's pickled skeleton


def _tag(epoch: int, b: int) -> int:
    return (epoch << 32) | (b + 1)


def _worker(w: int, conn, ring: SlotRing, epoch_word, dataset, rev_offset: RevOffset) -> None:
    torch.set_num_threads(1)
    flags, ep = ring.flags.numpy(), epoch_word.numpy()
    K = ring.per_worker
    while True:
        msg = conn.recv()
        if msg is None:
            return
        epoch, order = msg
        for s in range(w * K, (w + 1) * K):  # slots still tagged by an abandoned epoch
            flags[s] = 0
        for k, (b, sel) in enumerate(order):
            if ep[0] != epoch:
                break
            s = w * K + k % K
            while flags[s] != 0 and ep[0] == epoch:
                time.sleep(2e-5)
            if ep[0] != epoch:
                break
            try:
                graphs = dataset[sel.start:sel.stop] if isinstance(sel, slice) else [dataset[i] for i in sel]
                slot = ring.slot(s)
                data = slot[:ring.slot_bytes - META_BYTES]
                G = BatchedGraph.from_graphs(graphs, rev_offset, out=data)
                if 0 < G.packed_nbytes() <= data.numel():
                    blob = SlotBatch.pack(G, ring, s, out=data).blob
                    if len(blob) <= META_BYTES - 8:
                        meta = slot[ring.slot_bytes - META_BYTES:].numpy()
                        meta[:8] = np.frombuffer(len(blob).to_bytes(8, "little"), dtype=np.uint8)
                        meta[8:8 + len(blob)] = np.frombuffer(blob, dtype=np.uint8)
                        if ep[0] == epoch:
                            flags[s] = _tag(epoch, b)
                        continue
                # spill: every tensor out of the slot, through the pipe
                base, end = slot.data_ptr(), slot.data_ptr() + slot.numel()
                G._apply(lambda t: t.clone() if base <= t.data_ptr() < end else t, G)
                conn.send(("batch", epoch, b, G))
                flags[s] = -_tag(epoch, b)
            except Exception as e:  # raised in the parent at this batch
                import traceback

                conn.send(("error", epoch, b, f"{type(e).__name__}: {e}\n{traceback.format_exc()}"))
                flags[s] = -_tag(epoch, b)
                break


class GraphFeeder:
    """Iterate a dataset of per-molecule Graphs as collated host batches (SlotBatch for a batch in
    its ring slot, BatchedGraph for one that spilled), in batch order; wrap in DevicePrefetcher
    (graph_loader does) to get device batches.  Same batches as
    ``DataLoader(dataset, batch_size, shuffle, collate_fn=GraphCollator(rev_offset), drop_last)``."""

    def __init__(self, dataset: Sequence[Graph], batch_size: int, num_workers: int = 8, slots_per_worker: int = 3,
                 rev_offset: RevOffset = "nodes", shuffle: bool = False, drop_last: bool = False,
                 generator: Optional[torch.Generator] = None, slot_bytes: Optional[int] = None):
        if num_workers < 1 or batch_size < 1:
            raise ValueError("GraphFeeder needs num_workers >= 1 and batch_size >= 1")
        self.dataset, self.batch_size, self.W, self.K = dataset, batch_size, num_workers, slots_per_worker
        self.rev_offset, self.shuffle, self.drop_last, self.generator = rev_offset, shuffle, drop_last, generator
        if slot_bytes is None:
            first = BatchedGraph.from_graphs([dataset[i] for i in range(min(batch_size, len(dataset)))], rev_offset)
            slot_bytes = first.packed_nbytes() * 3 // 2 + (1 << 16)
        self.ring = SlotRing(num_workers, slots_per_worker, slot_bytes + META_BYTES)
        self.epoch_word = torch.zeros(1, dtype=torch.int64).share_memory_()
        self.epoch = 0
        self.procs: list = []
        self.conns: list = []
        # called while the consumer polls for a batch: DevicePrefetcher frees the slots whose copies
        # finished (a worker may be waiting for one of them to write the very batch polled for)
        self.on_wait = None

    def __len__(self) -> int:
        n = len(self.dataset)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def _start(self) -> None:
        import multiprocessing as mp

        from notorch_amd import _lib

        _lib.load()  # the collate library before the fork
        ctx = mp.get_context("fork")
        for w in range(self.W):
            a, b = ctx.Pipe(duplex=True)
            p = ctx.Process(target=_worker, args=(w, b, self.ring, self.epoch_word, self.dataset, self.rev_offset),
                            daemon=True, name=f"nt_feed_{w}")
            p.start()
            b.close()
            self.procs.append(p)
            self.conns.append(a)
        self.ring.register()  # after the fork: the workers map the ring as plain shared memory

    def _order(self) -> list:
        n = len(self.dataset)
        if self.shuffle:
            perm = torch.randperm(n, generator=self.generator).tolist()
            sel = [perm[i:i + self.batch_size] for i in range(0, n, self.batch_size)]
        else:
            sel = [slice(i, min(i + self.batch_size, n)) for i in range(0, n, self.batch_size)]
        return sel[:len(self)]

    def __iter__(self):
        # not a generator: the workers fork (and the ring is page-locked) here, before the caller
        # touches the ring
        if not self.procs:
            self._start()
        self.epoch += 1
        epoch = self.epoch
        self.epoch_word.numpy()[0] = epoch
        order = self._order()
        for w, c in enumerate(self.conns):
            c.send((epoch, [(b, order[b]) for b in range(w, len(order), self.W)]))
        return self._batches(epoch, len(order))

    def _batches(self, epoch: int, nb: int):
        flags = self.ring.flags.numpy()
        for b in range(nb):
            w, k = b % self.W, b // self.W
            s = w * self.K + k % self.K
            tag = _tag(epoch, b)
            spins = 0
            while True:
                f = flags[s]
                if f == tag:
                    meta = self.ring.slot(s)[self.ring.slot_bytes - META_BYTES:].numpy()
                    n = int.from_bytes(meta[:8].tobytes(), "little")
                    yield SlotBatch(s, meta[8:8 + n].tobytes())
                    break
                if f == -tag:
                    while True:  # (messages of an abandoned epoch are dropped)
                        kind, ep, bb, payload = self.conns[w].recv()
                        if (ep, bb) == (epoch, b):
                            break
                    if kind == "error":
                        raise RuntimeError(f"GraphFeeder worker {w}, batch {b}: {payload}")
                    flags[s] = 0  # the batch came through the pipe: the slot is free again
                    yield payload
                    break
                spins += 1
                if self.on_wait is not None:
                    self.on_wait()
                if spins % 4096 == 0 and not self.procs[w].is_alive():
                    raise RuntimeError(f"GraphFeeder worker {w} died (exit code {self.procs[w].exitcode})")
                time.sleep(1e-5)

    def close(self) -> None:
        self.epoch_word.numpy()[0] = -1  # any worker mid-epoch stops
        for c in self.conns:
            try:
                c.send(None)
            except (OSError, BrokenPipeError):
                pass
        for p in self.procs:
            p.join(timeout=5)
            if p.is_alive():
                p.terminate()
        self.procs, self.conns = [], []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
