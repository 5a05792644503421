"""oracle/ — TEST INFRASTRUCTURE ONLY.

A CPU restatement of the reference (davidegraff/notorch @ 2025-02-20) bond-message D-MPNN path,
used solely as the checker by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg.  The product (``notorch_amd``) never imports it.

PARITY UNPINNED (by the reference itself): the reference cannot be imported in this environment
(it requires Python >= 3.12 / PEP 695 syntax and torch_scatter, rdkit, tensordict, lightning,
jaxtyping, hydra — SURVEY §8(c)), and its own tests hold no golden vectors for this path (they
only assert training-loss thresholds).  The restatement is therefore pinned by
hand-derived known-answer tests (diatomic closed form, hand-computed 3-atom chain / star /
triangle), an fp64 cross-check, and committed fixtures it generated (tests/golden/).

Modules:
  dmpnn_ref   torch (ATen CPU) restatement of chemprop.py / residual.py / agg.py + torch_scatter
  collate_ref pure-Python restatement of BatchedGraph.from_graphs (graph.py:186-223)
"""
