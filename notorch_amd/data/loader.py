"""Host feed for the device path: collate in DataLoader workers, pinned host
batches, asynchronous H2D on a side stream overlapped with the current step.

Reference path: ``NotorchDataset.collate`` (notorch/data/dataset.py:56-71) calls
``TransformManager.collate`` (notorch/data/managers.py:44-53), which for graph inputs is
``MolToGraph.collate = BatchedGraph.from_graphs`` (notorch/transforms/graph.py:45), run inside torch
DataLoader worker processes; Lightning then moves each batch to the device on the training stream.

Here:

* :class:`GraphCollator` is that collate (``BatchedGraph.from_graphs``: the native one-pass C++
  collate, which also ships the CSR layout and the fused tile plan), picklable for the workers.
  Workers are forked from the main process and only run host code (the library was loaded before
  the fork; a worker makes no HIP call).
* The collator packs every tensor of the batch (features, indices, CSR layout, tile plan) into one
  buffer (``Graph.pack``), allocated in shared memory inside a worker: one storage crosses the
  worker queue without a further copy, is pinned and is copied to the device, instead of ~15.
  The per-graph walk that feeds the native collate runs in C++ too (``csrc/host/collate_py.cpp``).
* ``BatchedGraph.pin_memory()`` runs on a small thread pool of the main process
  (``DevicePrefetcher(pin_threads=...)``; the DataLoader's own pin thread with ``pin_threads=0``).
* :class:`DevicePrefetcher` issues batch i+1's copies (``non_blocking``) on a side stream while the
  caller's stream computes on batch i; the caller's stream waits on the copy's event before it
  touches the batch, and every moved tensor is recorded on the caller's stream for the caching
  allocator.
"""
from __future__ import annotations

from typing import Iterable, Iterator, Optional, Sequence

import torch

from notorch_amd.data.models.graph import BatchedGraph, Graph, RevOffset


class GraphCollator:
    """``collate_fn`` for a dataset of per-molecule :class:`Graph` items (transforms/graph.py:45)."""

    def __init__(self, rev_offset: RevOffset = "nodes"):
        self.rev_offset = rev_offset

    def __call__(self, graphs: Sequence[Graph]) -> BatchedGraph:
        # one buffer per batch: one storage to ship to the main process, pin and copy to the device;
        # in a worker it is allocated in shared memory, where the worker queue would copy it anyway
        in_worker = torch.utils.data.get_worker_info() is not None
        return BatchedGraph.from_graphs(graphs, self.rev_offset).pack(shared=in_worker)


def pinned_in_order(batches: Iterable, threads: int, pin, device_index: Optional[int] = None) -> Iterator:
    """pin(b) for every b of `batches`, computed by `threads` threads, yielded in the input order.
    A feeder thread draws from `batches` (at most 2 x threads pins in flight); an exception of the
    source or of a pin is raised to the consumer at that batch's position."""
    import queue
    import threading
    from concurrent.futures import ThreadPoolExecutor

    init = (lambda: torch.cuda.set_device(device_index)) if device_index is not None else None
    pool = ThreadPoolExecutor(threads, initializer=init, thread_name_prefix="nt_pin")
    q: queue.Queue = queue.Queue(maxsize=2 * threads)
    stop = threading.Event()
    end = object()

    def feed():
        try:
            for b in batches:
                if stop.is_set():
                    return
                q.put(pool.submit(pin, b))
            q.put(end)
        except BaseException as e:  # the consumer re-raises it
            q.put(e)

    t = threading.Thread(target=feed, daemon=True, name="nt_pin_feed")
    t.start()
    try:
        while True:
            f = q.get()
            if f is end:
                return
            if isinstance(f, BaseException):
                raise f
            yield f.result()
    finally:
        stop.set()
        while t.is_alive():  # unblock a feeder waiting on a full queue
            try:
                q.get_nowait()
            except queue.Empty:
                t.join(timeout=0.01)
        pool.shutdown(wait=True)


class DevicePrefetcher:
    """Iterate host batches as device batches, one batch of H2D copies ahead of the consumer.

    pin_threads > 0: the host batches are pageable (DataLoader(pin_memory=False)); a feeder thread
    takes them from the loader in order and `pin_threads` threads pin them concurrently (each pin is
    a 7 MB copy out of the worker's shared-memory segment at config 2, which one pin thread -- the
    DataLoader's own -- cannot do at the device's rate).  Order is kept: batches come out as the
    loader yields them."""

    def __init__(self, batches: Iterable[BatchedGraph], device: torch.device | str, pin_threads: int = 0):
        self.batches = batches
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(self.device)
        self.pin_threads = pin_threads

    def _issue(self, it: Iterator[BatchedGraph]) -> Optional[tuple]:
        try:
            host = next(it)
        except StopIteration:
            return None
        with torch.cuda.stream(self.stream):
            dev = host.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return dev, ev

    def __iter__(self) -> Iterator[BatchedGraph]:
        if self.pin_threads > 0:
            idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
            it = pinned_in_order(self.batches, self.pin_threads, BatchedGraph.pin_memory, idx)
        else:
            it = iter(self.batches)
        nxt = self._issue(it)
        while nxt is not None:
            G, ev = nxt
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            buf = G._packed_base()  # the allocator must not reuse these before the consumer is done
            for t in ([buf] if buf is not None else G.tensors()):
                t.record_stream(cur)
            nxt = self._issue(it)  # the next batch's copies overlap this batch's compute
            yield G


def graph_loader(
    dataset: Sequence[Graph],
    batch_size: int,
    device: torch.device | str,
    *,
    num_workers: int = 4,
    rev_offset: RevOffset = "nodes",
    shuffle: bool = False,
    prefetch_factor: int = 2,
    pin_threads: int = 4,
    **kwargs,
) -> DevicePrefetcher:
    """DataLoader (workers collate) wrapped in a :class:`DevicePrefetcher` whose `pin_threads`
    threads pin the batches (0: the DataLoader's single pin thread)."""
    from notorch_amd import _lib

    _lib.load()  # load the collate library before the workers fork
    dl = torch.utils.data.DataLoader(
        dataset, batch_size=batch_size, shuffle=shuffle, collate_fn=GraphCollator(rev_offset),
        num_workers=num_workers, pin_memory=pin_threads == 0, persistent_workers=num_workers > 0,
        prefetch_factor=prefetch_factor if num_workers > 0 else None, **kwargs,
    )
    return DevicePrefetcher(dl, device, pin_threads=pin_threads)
