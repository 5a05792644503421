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
* ``pin_memory=True`` makes the DataLoader's pin thread call ``BatchedGraph.pin_memory()``.
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


class DevicePrefetcher:
    """Iterate host batches as device batches, one batch of H2D copies ahead of the consumer."""

    def __init__(self, batches: Iterable[BatchedGraph], device: torch.device | str):
        self.batches = batches
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(self.device)

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
    **kwargs,
) -> DevicePrefetcher:
    """DataLoader (workers collate, pin thread pins) wrapped in a :class:`DevicePrefetcher`."""
    from notorch_amd import _lib

    _lib.load()  # load the collate library before the workers fork
    dl = torch.utils.data.DataLoader(
        dataset, batch_size=batch_size, shuffle=shuffle, collate_fn=GraphCollator(rev_offset),
        num_workers=num_workers, pin_memory=True, persistent_workers=num_workers > 0,
        prefetch_factor=prefetch_factor if num_workers > 0 else None, **kwargs,
    )
    return DevicePrefetcher(dl, device)
