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
  caller's stream computes on batch i (from a thread of its own by default, so that receiving and
  issuing a batch does not delay the caller's kernel launches); the caller's stream waits on the
  copy's event before it touches the batch, and every moved tensor is recorded on the caller's
  stream for the caching allocator.
* :class:`SlotRing` (the default with workers): page-locked shared-memory slots the workers
  collate straight into; a batch crosses the worker queue as a few KB of offsets and goes to the
  device by DMA from the slot, which is reused once that copy has completed.
"""
from __future__ import annotations

from typing import Iterable, Iterator, Optional, Sequence

import torch

from notorch_amd.data.models.graph import BatchedGraph, Graph, RevOffset


class SlotRing:
    """Fixed shared-memory batch slots that DataLoader workers pack into, mapped once by every process.

    Created in the main process before the workers fork (they inherit the mapping); the main process
    then page-locks the whole ring once (``hipHostRegister``), so a batch goes from the worker's pack
    straight to the device by DMA: no per-batch shared-memory segment, file-descriptor hand-off,
    mapping, pinned copy or unmapping in the main process.  Worker w owns slots
    [w * per_worker, (w + 1) * per_worker); ``flags[s]`` is 1 from the worker's pack until the main
    process's copy out of slot s has completed."""

    def __init__(self, workers: int, per_worker: int, slot_bytes: int):
        self.workers, self.per_worker = workers, per_worker
        self.slot_bytes = (slot_bytes + 63) // 64 * 64
        n = workers * per_worker
        self.buf = torch.empty(0, dtype=torch.uint8).set_(
            torch.UntypedStorage._new_shared(n * self.slot_bytes), 0, (n * self.slot_bytes,), (1,))
        self.flags = torch.zeros(n, dtype=torch.int64).share_memory_()
        self.registered = False

    def slot(self, s: int) -> torch.Tensor:
        return self.buf[s * self.slot_bytes:(s + 1) * self.slot_bytes]

    def acquire(self, worker: int, timeout_s: float = 2.0) -> int:
        """A free slot of `worker` (marked in use), or -1 after timeout_s (the caller then ships the
        batch the ordinary way)."""
        import time

        f = self.flags.numpy()
        t_end = time.monotonic() + timeout_s
        while True:
            for s in range(worker * self.per_worker, (worker + 1) * self.per_worker):
                if f[s] == 0:
                    f[s] = 1
                    return s
            if time.monotonic() > t_end:
                return -1
            time.sleep(5e-5)

    def release(self, s: int) -> None:
        self.flags.numpy()[s] = 0

    def register(self) -> bool:
        """Page-lock the ring for DMA (main process, after the workers forked)."""
        if not self.registered and torch.cuda.is_available():
            rc = torch.cuda.cudart().cudaHostRegister(self.buf.data_ptr(), self.buf.numel(), 0)
            self.registered = int(rc) == 0
        return self.registered

    def unregister(self) -> None:
        if self.registered:
            torch.cuda.cudart().cudaHostUnregister(self.buf.data_ptr())
            self.registered = False

    def __del__(self):
        try:
            self.unregister()
        except Exception:  # interpreter shutdown: the runtime may be gone
            pass

    @staticmethod
    def fits(nbytes: int) -> bool:
        """Whether /dev/shm has room for nbytes twice over (tmpfs raises SIGBUS on a page past its
        limit, so the ring is only used when it fits with margin)."""
        import os

        try:
            st = os.statvfs("/dev/shm")
        except OSError:
            return False
        return st.f_bavail * st.f_frsize >= 2 * nbytes


class SlotBatch:
    """What a worker returns for a batch packed into ring slot `slot`: the batch pickled with every
    tensor inside the slot replaced by its (offset, dtype, shape, stride): a few KB through the
    worker queue instead of a shared-memory segment."""

    __slots__ = ("slot", "blob")

    def __init__(self, slot: int, blob: bytes):
        self.slot, self.blob = slot, blob

    @staticmethod
    def pack(G: BatchedGraph, ring: SlotRing, s: int, out: Optional[torch.Tensor] = None) -> "SlotBatch":
        """out: the part of slot s to pack into (default: all of it)."""
        import io
        import pickle

        G.pack(out=ring.slot(s) if out is None else out)
        base = ring.slot(s).data_ptr()
        end = base + ring.slot_bytes

        class P(pickle.Pickler):
            def persistent_id(self, obj):
                if isinstance(obj, torch.Tensor) and obj.device.type == "cpu" and base <= obj.data_ptr() < end:
                    return ("nt_slot", obj.data_ptr() - base, obj.dtype, tuple(obj.shape), tuple(obj.stride()))
                return None

        f = io.BytesIO()
        P(f, pickle.HIGHEST_PROTOCOL).dump(G)
        return SlotBatch(s, f.getvalue())

    def load(self, ring: SlotRing) -> BatchedGraph:
        import io
        import pickle

        storage = ring.buf.untyped_storage()
        off0 = self.slot * ring.slot_bytes

        class U(pickle.Unpickler):
            def persistent_load(self, pid):
                _, off, dtype, shape, stride = pid
                isz = torch.empty(0, dtype=dtype).element_size()
                return torch.empty(0, dtype=dtype).set_(storage, (off0 + off) // isz, shape, stride)

        return U(io.BytesIO(self.blob)).load()


class GraphCollator:
    """``collate_fn`` for a dataset of per-molecule :class:`Graph` items (transforms/graph.py:45).
    ring: pack worker batches into its slots (graph_loader sets it); None: one shared-memory buffer
    per batch."""

    def __init__(self, rev_offset: RevOffset = "nodes", ring: Optional[SlotRing] = None):
        self.rev_offset = rev_offset
        self.ring = ring

    def __call__(self, graphs: Sequence[Graph]):
        # one buffer per batch: one storage to ship to the main process, pin and copy to the device;
        # in a worker it is allocated in shared memory, where the worker queue would copy it anyway
        info = torch.utils.data.get_worker_info()
        s = self.ring.acquire(info.id) if info is not None and self.ring is not None else -1
        if s < 0:
            return BatchedGraph.from_graphs(graphs, self.rev_offset).pack(shared=info is not None)
        # the collate writes straight into the slot; pack() then copies only the layout's plans
        slot = self.ring.slot(s)
        G = BatchedGraph.from_graphs(graphs, self.rev_offset, out=slot)
        if 0 < G.packed_nbytes() <= self.ring.slot_bytes:
            return SlotBatch.pack(G, self.ring, s)
        # does not fit (or does not pack): move every tensor out of the slot, then free it
        base, end = slot.data_ptr(), slot.data_ptr() + slot.numel()
        G._apply(lambda t: t.clone() if base <= t.data_ptr() < end else t, G)
        self.ring.release(s)
        return G.pack(shared=True)


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


def _pin(b):
    return b if isinstance(b, SlotBatch) else BatchedGraph.pin_memory(b)


class DevicePrefetcher:
    """Iterate host batches as device batches, one batch of H2D copies ahead of the consumer.

    pin_threads > 0: the host batches are pageable (DataLoader(pin_memory=False)); a feeder thread
    takes them from the loader in order and `pin_threads` threads pin them concurrently (each pin is
    a 7 MB copy out of the worker's shared-memory segment at config 2, which one pin thread -- the
    DataLoader's own -- cannot do at the device's rate).  Order is kept: batches come out as the
    loader yields them."""

    def __init__(self, batches: Iterable[BatchedGraph], device: torch.device | str, pin_threads: int = 0,
                 ring: Optional[SlotRing] = None, background: bool = False):
        self.batches = batches
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(self.device)
        self.pin_threads = pin_threads
        self.ring = ring
        self.background = background
        self._held: list = []  # (event, slot): ring slots whose device copy may still be running
        if ring is not None and hasattr(batches, "on_wait"):
            batches.on_wait = self._release_done

    def _release_done(self, wait: bool = False) -> None:
        keep = []
        for ev, s in self._held:
            if wait:
                ev.synchronize()
            if wait or ev.query():
                self.ring.release(s)
            else:
                keep.append((ev, s))
        self._held = keep

    def _issue(self, it: Iterator[BatchedGraph]) -> Optional[tuple]:
        if self._held:
            self._release_done()  # before blocking on the loader: a worker may be waiting for a slot
        try:
            host = next(it)
        except StopIteration:
            return None
        slot = -1
        if isinstance(host, SlotBatch):
            slot, host = host.slot, host.load(self.ring)
            if not self.ring.registered:  # no page-locked ring: copy out into pinned memory first
                pinned = host.pin_memory()
                self.ring.release(slot)
                slot, host = -1, pinned
        elif self.ring is not None:  # a batch that missed a slot (no DataLoader pin thread here)
            host = host.pin_memory()
        with torch.cuda.stream(self.stream):
            dev = host.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        if slot >= 0:
            self._held.append((ev, slot))
        return dev, ev

    def __iter__(self) -> Iterator[BatchedGraph]:
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        if self.pin_threads > 0:
            it = pinned_in_order(self.batches, self.pin_threads, _pin, idx)
        else:
            it = iter(self.batches)  # (forks the DataLoader's workers: the ring is registered after)
        if self.ring is not None:
            self.ring.register()
        src = self._background(it, idx) if self.background else self._inline(it)
        try:
            for G, ev in src:
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(ev)
                buf = G._packed_base()  # the allocator must not reuse these before the consumer is done
                for t in ([buf] if buf is not None else G.tensors()):
                    t.record_stream(cur)
                yield G
        finally:
            src.close()
            if self.ring is not None:
                self._release_done(wait=True)

    def _inline(self, it):
        nxt = self._issue(it)
        while nxt is not None:
            cur = nxt
            nxt = self._issue(it)  # the next batch's copies overlap this batch's compute
            yield cur

    def _background(self, it, idx: int):
        """_issue on a thread of its own, two batches ahead: the consumer thread only waits on a queue,
        so its kernel launches do not queue behind the loader's bookkeeping and the H2D issue."""
        import queue
        import threading

        q: queue.Queue = queue.Queue(maxsize=2)
        stop = threading.Event()
        end = object()

        def produce():
            torch.cuda.set_device(idx)
            try:
                while not stop.is_set():
                    nxt = self._issue(it)
                    q.put(end if nxt is None else nxt)
                    if nxt is None:
                        return
            except BaseException as e:  # re-raised by the consumer
                q.put(e)

        t = threading.Thread(target=produce, daemon=True, name="nt_h2d_feed")
        t.start()
        try:
            while True:
                item = q.get()
                if item is end:
                    return
                if isinstance(item, BaseException):
                    raise item
                yield item
        finally:
            stop.set()
            while t.is_alive():  # unblock a producer waiting on a full queue
                try:
                    q.get_nowait()
                except queue.Empty:
                    t.join(timeout=0.01)


def graph_loader(
    dataset: Sequence[Graph],
    batch_size: int,
    device: torch.device | str,
    *,
    num_workers: int = 4,
    rev_offset: RevOffset = "nodes",
    shuffle: bool = False,
    prefetch_factor: int = 2,
    pin_threads: int = 0,
    ring_slots: int = 3,
    background: bool = False,
    feeder: bool = True,
    generator: Optional[torch.Generator] = None,
    drop_last: bool = False,
    **kwargs,
) -> DevicePrefetcher:
    """DataLoader (workers collate) wrapped in a :class:`DevicePrefetcher`.

    ring_slots > 0 (and workers): batches travel through a page-locked :class:`SlotRing` of
    `ring_slots` slots per worker, sized from the first batch (x 1.5); a batch that does not fit, or
    finds no free slot, takes the path below.  Otherwise each batch is one shared-memory buffer, pinned
    by the DataLoader's pin thread (pin_threads = 0) or by `pin_threads` threads of the main process.
    background: receive batches and issue their H2D copies on a thread of the prefetcher's own.
    feeder (with workers and ring slots, no other DataLoader arguments): the DataLoader-free
    :class:`notorch_amd.data.feeder.GraphFeeder` instead of a torch DataLoader."""
    from notorch_amd import _lib

    _lib.load()  # load the collate library before the workers fork
    if feeder and ring_slots > 0 and num_workers > 0 and not kwargs and len(dataset) > 0 and torch.cuda.is_available():
        from notorch_amd.data.feeder import META_BYTES, GraphFeeder

        first = BatchedGraph.from_graphs([dataset[i] for i in range(min(batch_size, len(dataset)))], rev_offset)
        slot = first.packed_nbytes() * 3 // 2 + (1 << 16)
        if first.packed_nbytes() > 0 and SlotRing.fits(num_workers * ring_slots * (slot + META_BYTES)):
            f = GraphFeeder(dataset, batch_size, num_workers, ring_slots, rev_offset, shuffle, drop_last, generator,
                            slot_bytes=slot)
            return DevicePrefetcher(f, device, ring=f.ring, background=background)
    ring = None
    if ring_slots > 0 and num_workers > 0 and len(dataset) > 0 and torch.cuda.is_available():
        first = BatchedGraph.from_graphs([dataset[i] for i in range(min(batch_size, len(dataset)))], rev_offset)
        slot = first.packed_nbytes() * 3 // 2 + (1 << 16)
        if first.packed_nbytes() > 0 and SlotRing.fits(num_workers * ring_slots * slot):
            ring = SlotRing(num_workers, ring_slots, slot)
    coll = GraphCollator(rev_offset, ring)
    common = dict(num_workers=num_workers, persistent_workers=num_workers > 0,
                  prefetch_factor=prefetch_factor if num_workers > 0 else None, collate_fn=coll)
    # with the ring, batches arrive page-locked (a batch that missed a slot is pinned in _issue): no
    # DataLoader pin thread, whose hand-off costs the consumer thread time per batch
    pin = pin_threads == 0 and ring is None
    if not shuffle and not drop_last and not kwargs and isinstance(dataset, (list, tuple)):
        # sequential batches as slices: the index queue carries one range per batch instead of
        # batch_size ints, and a worker fetches its graphs with one slice
        dl = torch.utils.data.DataLoader(_Slices(dataset, batch_size), batch_size=None, pin_memory=pin, **common)
    else:
        dl = torch.utils.data.DataLoader(dataset, batch_size=batch_size, shuffle=shuffle, pin_memory=pin, **common,
                                         generator=generator, drop_last=drop_last, **kwargs)
    return DevicePrefetcher(dl, device, pin_threads=pin_threads, ring=ring, background=background)


class _Slices(torch.utils.data.Dataset):
    """Batch b of a list dataset = its b-th slice of batch_size items (the last one shorter)."""

    def __init__(self, data, batch_size: int):
        self.data, self.batch_size = data, batch_size

    def __len__(self) -> int:
        return (len(self.data) + self.batch_size - 1) // self.batch_size

    def __getitem__(self, b: int):
        return self.data[b * self.batch_size:(b + 1) * self.batch_size]
