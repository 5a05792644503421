"""Seeded synthetic molecule-shaped batches: QM9-, ZINC- and polymer-shaped graphs.

rdkit is not available, so the featurisation (``MolToGraph`` + ``MultiType{Atom,Bond}Transform``)
is replaced by random type indices drawn per column inside the reference's vocab ranges
(atom column sizes [11,7,5,5,6,6,2] = 42 types, bond [5,8] = 13; notorch/transforms/conf.py,
atom.py:68-84, bond.py:48-58) on a random molecular topology.  The per-molecule layout is
exactly ``MolToGraph.__call__`` (notorch/transforms/graph.py:32-43): bond b -> directed edges
2b = (u->v) and 2b+1 = (v->u); ``rev_index = [1, 0, 3, 2, ...]``; bond features repeated twice.

Generators (numpy ``default_rng(seed)``):
* qm9:     n_atoms in {9, 8, 7} w.p. {.90, .08, .02}; random spanning tree with max degree 4,
           plus {0,1,2,3} ring closures w.p. {.15, .30, .35, .20}.
* zinc:    n_atoms = round(N(23.2, 4.5)) clipped to [6, 38]; tree + Poisson(2.7) ring closures.
* polymer: n ~ U[1000, 10000]; backbone chain + short branches (degree <= 4), plus 0.5 % hub
           atoms with extra bonds up to degree ~ U[16, 512] (segment-length skew stress).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Literal

import numpy as np
import torch

ATOM_TYPE_SIZES = (11, 7, 5, 5, 6, 6, 2)
BOND_TYPE_SIZES = (5, 8)
DEFAULT_NUM_ATOM_TYPES = sum(ATOM_TYPE_SIZES)  # 42
DEFAULT_NUM_BOND_TYPES = sum(BOND_TYPE_SIZES)  # 13

Kind = Literal["qm9", "zinc", "polymer"]


def _tree(rng: np.random.Generator, n: int, max_deg: int = 4) -> tuple[list, np.ndarray]:
    deg = np.zeros(n, dtype=np.int64)
    bonds = []
    for i in range(1, n):
        cand = np.flatnonzero(deg[:i] < max_deg)
        j = int(cand[rng.integers(len(cand))])
        bonds.append((j, i))
        deg[i] += 1
        deg[j] += 1
    return bonds, deg


def _add_rings(rng, n, bonds, deg, k, max_deg=4, tries=30):
    present = {(min(u, v), max(u, v)) for u, v in bonds}
    added = 0
    for _ in range(tries):
        if added >= k:
            break
        u, v = (int(x) for x in rng.integers(n, size=2))
        if u == v or deg[u] >= max_deg or deg[v] >= max_deg:
            continue
        key = (min(u, v), max(u, v))
        if key in present:
            continue
        present.add(key)
        bonds.append((u, v))
        deg[u] += 1
        deg[v] += 1
        added += 1
    return bonds


def _qm9_mol(rng):
    n = int(rng.choice([9, 8, 7], p=[0.90, 0.08, 0.02]))
    bonds, deg = _tree(rng, n)
    k = int(rng.choice([0, 1, 2, 3], p=[0.15, 0.30, 0.35, 0.20]))
    return n, _add_rings(rng, n, bonds, deg, k)


def _zinc_mol(rng):
    n = int(np.clip(round(rng.normal(23.2, 4.5)), 6, 38))
    bonds, deg = _tree(rng, n)
    return n, _add_rings(rng, n, bonds, deg, int(rng.poisson(2.7)))


def _polymer_mol(rng):
    n = int(rng.integers(1000, 10001))
    L = max(2, int(0.6 * n))
    bonds = [(i, i + 1) for i in range(L - 1)]
    deg = np.zeros(n, dtype=np.int64)
    deg[: L - 1] += 1
    deg[1:L] += 1
    for i in range(L, n):  # short branches: attach to a random earlier atom with free valence
        for _ in range(50):
            j = int(rng.integers(i))
            if deg[j] < 4:
                break
        bonds.append((j, i))
        deg[i] += 1
        deg[j] += 1
    present = {(min(u, v), max(u, v)) for u, v in bonds}
    n_hubs = max(1, int(round(0.005 * n)))
    for hub in rng.choice(n, size=n_hubs, replace=False):
        hub = int(hub)
        target = min(int(rng.integers(16, 513)), n - 1)
        partners = rng.permutation(n)
        for p in partners:
            if deg[hub] >= target:
                break
            p = int(p)
            key = (min(hub, p), max(hub, p))
            if p == hub or key in present:
                continue
            present.add(key)
            bonds.append((p, hub))
            deg[hub] += 1
            deg[p] += 1
    return n, bonds


_GEN = {"qm9": _qm9_mol, "zinc": _zinc_mol, "polymer": _polymer_mol}


@dataclass
class SynthMolBatch:
    """Flat description of B molecules.  ``bonds`` holds LOCAL atom ids, molecule after molecule."""

    n_atoms: np.ndarray  # (B,)
    n_bonds: np.ndarray  # (B,)
    bonds: np.ndarray  # (Nb, 2) int64, local ids
    atom_types: np.ndarray  # (V, 7) int64
    bond_types: np.ndarray  # (Nb, 2) int64

    @property
    def num_graphs(self) -> int:
        return len(self.n_atoms)

    @property
    def num_nodes(self) -> int:
        return int(self.n_atoms.sum())

    @property
    def num_edges(self) -> int:
        return int(2 * self.n_bonds.sum())

    def subset(self, start: int, stop: int) -> "SynthMolBatch":
        """Molecules [start, stop) (contiguous shard)."""
        a0, a1 = int(self.n_atoms[:start].sum()), int(self.n_atoms[:stop].sum())
        b0, b1 = int(self.n_bonds[:start].sum()), int(self.n_bonds[:stop].sum())
        return SynthMolBatch(
            self.n_atoms[start:stop].copy(),
            self.n_bonds[start:stop].copy(),
            self.bonds[b0:b1].copy(),
            self.atom_types[a0:a1].copy(),
            self.bond_types[b0:b1].copy(),
        )

    # ---- per-molecule graphs in MolToGraph layout (transforms/graph.py:32-43) ----
    def to_graphs(self):
        from notorch_amd.data.models.graph import Graph

        Gs = []
        a0 = b0 = 0
        for n, nb in zip(self.n_atoms.tolist(), self.n_bonds.tolist()):
            bonds = self.bonds[b0 : b0 + nb]
            V = torch.from_numpy(self.atom_types[a0 : a0 + n].copy())
            E = torch.from_numpy(self.bond_types[b0 : b0 + nb].copy()).repeat_interleave(2, dim=0)
            ei = np.empty((2, 2 * nb), dtype=np.int64)
            ei[0, 0::2], ei[1, 0::2] = bonds[:, 0], bonds[:, 1]
            ei[0, 1::2], ei[1, 1::2] = bonds[:, 1], bonds[:, 0]
            rev = np.arange(2 * nb).reshape(-1, 2)[:, ::-1].ravel().copy()
            Gs.append(Graph(V, E, torch.from_numpy(ei), torch.from_numpy(rev)))
            a0 += n
            b0 += nb
        return Gs

    # ---- vectorised collate straight from the flat arrays (== from_graphs(to_graphs())) ----
    def collate(self, rev_offset: str = "nodes"):
        from notorch_amd.data.models.graph import BatchedGraph, host_layout

        B = self.num_graphs
        node_off = np.cumsum(self.n_atoms) - self.n_atoms
        edge_off = 2 * (np.cumsum(self.n_bonds) - self.n_bonds)
        mol_of_bond = np.repeat(np.arange(B), self.n_bonds)
        u = self.bonds[:, 0] + node_off[mol_of_bond]
        v = self.bonds[:, 1] + node_off[mol_of_bond]
        Ne = 2 * len(self.bonds)
        ei = np.empty((2, Ne), dtype=np.int64)
        ei[0, 0::2], ei[1, 0::2] = u, v
        ei[0, 1::2], ei[1, 1::2] = v, u
        mol_of_edge = np.repeat(np.arange(B), 2 * self.n_bonds)
        local = np.arange(Ne) - edge_off[mol_of_edge]
        base = node_off if rev_offset == "nodes" else edge_off
        rev = (local ^ 1) + base[mol_of_edge]
        edge_index = torch.from_numpy(ei)
        rev_index = torch.from_numpy(rev.astype(np.int64))
        bni = torch.from_numpy(np.repeat(np.arange(B), self.n_atoms).astype(np.int64))
        bei = torch.from_numpy(mol_of_edge.astype(np.int64))
        BG = BatchedGraph(
            torch.from_numpy(self.atom_types),
            torch.from_numpy(np.repeat(self.bond_types, 2, axis=0)),
            edge_index,
            rev_index,
            batch_node_index=bni,
            batch_edge_index=bei,
            size=B,
        )
        BG._nt_layout = host_layout(edge_index, rev_index, self.num_nodes, bni, B, BG.node_feats,
                                    BG.edge_feats)
        return BG


def _types(rng: np.random.Generator, V: int, Nb: int) -> tuple[np.ndarray, np.ndarray]:
    a_off = np.cumsum((0,) + ATOM_TYPE_SIZES[:-1])
    b_off = np.cumsum((0,) + BOND_TYPE_SIZES[:-1])
    atom_types = np.stack(
        [o + rng.integers(s, size=V) for o, s in zip(a_off, ATOM_TYPE_SIZES)], axis=1
    ).astype(np.int64)
    bond_types = np.stack(
        [o + rng.integers(s, size=Nb) for o, s in zip(b_off, BOND_TYPE_SIZES)], axis=1
    ).astype(np.int64).reshape(Nb, 2)
    return atom_types, bond_types


def make_qm9_batch_vectorized(num_mols: int, seed: int = 0, ring_tries: int = 30) -> SynthMolBatch:
    """The QM9 generator of ``make_batch("qm9", ...)`` vectorised over molecules (same
    distribution, a different random stream), for million-molecule batches (BASELINE config 4):
    every step draws for all molecules at once.

    * n_atoms in {9, 8, 7} w.p. {.90, .08, .02};
    * spanning tree: atom i (1 <= i < n) bonds to a uniformly drawn earlier atom of degree < 4;
    * ring closures: k in {0,1,2,3} w.p. {.15, .30, .35, .20}; up to ``ring_tries`` draws of a
      random atom pair, accepted while fewer than k were added, u != v, both degrees < 4 and the
      pair not bonded yet.
    Bonds of a molecule are listed tree bonds first (in atom order), then ring closures."""
    rng = np.random.default_rng(seed)
    B = int(num_mols)
    N = 9
    n = rng.choice(np.array([9, 8, 7]), size=B, p=[0.90, 0.08, 0.02]).astype(np.int64)
    deg = np.zeros((B, N), dtype=np.int64)
    adj = np.zeros((B, N, N), dtype=bool)
    rows = np.arange(B)
    cand_u = np.zeros((B, N - 1 + ring_tries), dtype=np.int64)
    cand_v = np.zeros((B, N - 1 + ring_tries), dtype=np.int64)
    keep = np.zeros((B, N - 1 + ring_tries), dtype=bool)
    for i in range(1, N):
        active = i < n
        scores = rng.random((B, i))
        scores[deg[:, :i] >= 4] = -1.0
        j = scores.argmax(1)
        cand_u[:, i - 1], cand_v[:, i - 1], keep[:, i - 1] = j, i, active
        a = rows[active]
        deg[a, j[active]] += 1
        deg[a, i] += 1
        adj[a, j[active], i] = adj[a, i, j[active]] = True
    k = rng.choice(np.array([0, 1, 2, 3]), size=B, p=[0.15, 0.30, 0.35, 0.20])
    added = np.zeros(B, dtype=np.int64)
    for t in range(ring_tries):
        u = rng.integers(0, n)
        v = rng.integers(0, n)
        ok = (added < k) & (u != v) & (deg[rows, u] < 4) & (deg[rows, v] < 4) & ~adj[rows, u, v]
        c = N - 1 + t
        cand_u[:, c], cand_v[:, c], keep[:, c] = u, v, ok
        a = rows[ok]
        deg[a, u[ok]] += 1
        deg[a, v[ok]] += 1
        adj[a, u[ok], v[ok]] = adj[a, v[ok], u[ok]] = True
        added += ok
    n_bonds = keep.sum(1).astype(np.int64)
    bonds = np.stack([cand_u[keep], cand_v[keep]], axis=1).astype(np.int64)
    atom_types, bond_types = _types(rng, int(n.sum()), len(bonds))
    return SynthMolBatch(n, n_bonds, bonds, atom_types, bond_types)


def make_batch(kind: Kind, num_mols: int, seed: int = 0) -> SynthMolBatch:
    rng = np.random.default_rng(seed)
    gen = _GEN[kind]
    n_atoms, n_bonds, bonds = [], [], []
    for _ in range(num_mols):
        n, bl = gen(rng)
        n_atoms.append(n)
        n_bonds.append(len(bl))
        bonds.extend(bl)
    n_atoms = np.asarray(n_atoms, dtype=np.int64)
    n_bonds = np.asarray(n_bonds, dtype=np.int64)
    bonds_arr = np.asarray(bonds, dtype=np.int64).reshape(-1, 2)
    atom_types, bond_types = _types(rng, int(n_atoms.sum()), len(bonds_arr))
    return SynthMolBatch(n_atoms, n_bonds, bonds_arr, atom_types, bond_types)
