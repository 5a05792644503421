"""hipGraph capture of a whole forward (PyTorch's ``torch.cuda.CUDAGraph`` is a hipGraph on ROCm).

The notorch_amd kernels are stream-ordered, allocate nothing themselves and launch on
``torch.cuda.current_stream()``, so a forward (``ChempropBlock`` + readout, or the embedded encoder)
can be captured once and replayed with one host call: for small batches (SURVEY §8(d) config 1,
32 molecules) the d + 2 kernel launches and the Python around them dominate, and a replay removes
both.  The first (eager) calls build and cache everything that needs the host — the CSR layout and
its validation, the fused tile plan, chunk plans and packed weights — so nothing synchronises
inside the capture.

Usage::

    fwd = GraphedForward(lambda G: readout(block(G)), G)   # warm-up + capture on G's device
    out = fwd()                                            # replay on the same input buffers
    fwd.copy_inputs(G2)                                    # same shapes: refill the static inputs

A replay recomputes every kernel of the captured forward on whatever the static input buffers hold;
it is a launch-overhead optimisation, not a cache.
"""
from __future__ import annotations

from typing import Any, Callable

import torch

__all__ = ["GraphedForward"]


class GraphedForward:
    def __init__(self, fn: Callable[[Any], Any], G, warmup: int = 2):
        dev = G.node_feats.device
        if dev.type != "cuda":
            raise RuntimeError("GraphedForward needs a graph on a ROCm device")
        self.fn, self.G = fn, G
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.no_grad(), torch.cuda.stream(side):
            for _ in range(max(1, warmup)):  # builds + caches layouts, plans, packed weights
                fn(G)
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(self.graph):
            self.out = fn(G)

    def __call__(self):
        self.graph.replay()
        return self.out

    def copy_inputs(self, G) -> None:
        """Refill the captured input buffers from a graph with identical shapes and topology
        (features can change freely; a different topology needs a new capture, since the CSR and
        tile plan of the captured graph are baked into the replay)."""
        for f in ("node_feats", "edge_feats"):
            dst, src = getattr(self.G, f), getattr(G, f)
            if dst.shape != src.shape or dst.dtype != src.dtype:
                raise ValueError(f"{f}: shape/dtype {tuple(src.shape)}/{src.dtype} differs from the "
                                 f"captured {tuple(dst.shape)}/{dst.dtype}")
            dst.copy_(src, non_blocking=True)
