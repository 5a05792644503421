"""Generate the committed golden fixtures under tests/golden/ (run from the repo root:
``python tests/golden/make_golden.py``).

The reference cannot run in this environment, so the expected outputs come from
the CPU restatement in oracle/dmpnn_ref.py (ATen CPU kernels, fp32), cross-checked against an
fp64 evaluation of the same restatement (stored too).  Inputs are seeded synthetic QM9-shaped
molecules collated with the reference collate semantics (rev offset by nodes, graph.py:200).

Fixtures:
  config1.npz  32 QM9-shaped molecules, h=300, depth=3, ReLU, residual, sum (BASELINE config 1)
  tiny.npz     4 molecules, h=16, depth=2, same options (fast KAT-sized case)
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from notorch_amd.data.synth import make_batch  # noqa: E402
from oracle import dmpnn_ref  # noqa: E402


def build(num_mols: int, h: int, depth: int, seed: int) -> dict:
    torch.manual_seed(seed)
    batch = make_batch("qm9", num_mols, seed=seed)
    G = batch.collate("nodes")
    node_tab = torch.nn.EmbeddingBag(42, h, mode="sum")
    edge_tab = torch.nn.EmbeddingBag(13, h, mode="sum")
    with torch.no_grad():
        Xv = node_tab(G.node_feats)
        Xe = edge_tab(G.edge_feats)
        lins = [torch.nn.Linear(h, h) for _ in range(depth)]
        W = [lin.weight.detach().clone() for lin in lins]
        b = [lin.bias.detach().clone() for lin in lins]
        node, edge = dmpnn_ref.chemprop_block(Xv, Xe, G.edge_index, G.rev_index, W, b)
        out = dmpnn_ref.readout(node, G.batch_node_index, len(G), "sum")
        node64, edge64 = dmpnn_ref.chemprop_block(
            Xv.double(), Xe.double(), G.edge_index, G.rev_index, [w.double() for w in W], [x.double() for x in b]
        )
        out64 = dmpnn_ref.readout(node64, G.batch_node_index, len(G), "sum")
    return dict(
        node_feats=Xv.numpy(), edge_feats=Xe.numpy(), edge_index=G.edge_index.numpy(),
        rev_index=G.rev_index.numpy(), batch_node_index=G.batch_node_index.numpy(),
        batch_edge_index=G.batch_edge_index.numpy(), size=np.int64(len(G)),
        atom_types=batch.atom_types, bond_types=batch.bond_types,
        W=torch.stack(W).numpy(), b=torch.stack(b).numpy(),
        out_node=node.numpy(), out_edge=edge.numpy(), out_sum=out.numpy(),
        out_sum64=out64.numpy(),
        # fp32 restatement vs fp64 truth (the noise floor any fp32 implementation sits on)
        err64_node=np.float64((node.double() - node64).abs().max()),
        err64_edge=np.float64((edge.double() - edge64).abs().max()),
    )


if __name__ == "__main__":
    here = os.path.dirname(os.path.abspath(__file__))
    np.savez_compressed(os.path.join(here, "config1.npz"), **build(32, 300, 3, seed=1))
    np.savez_compressed(os.path.join(here, "tiny.npz"), **build(4, 16, 2, seed=2))
    print("wrote config1.npz, tiny.npz")
