"""BASELINE config 4 on one GPU: the 125k-molecule shard rank 0 gets when ONE seeded 1M-molecule
QM9 batch is cut into 8 edge-balanced contiguous shards (shard.edge_balanced_ranges).

* fixed rev mode (rev offset by edges): the shard's forward (ChempropBlock + Sum,
  chemprop.py:81-88 / agg.py:23-29) equals, bit for bit, the concatenation of the forwards of its
  four edge-balanced sub-batches — what the per-GPU sub-batches of config 4 compute;
* compat rev mode (the reference collate, graph.py:200): the full shard runs, deterministically,
  and sampled 64-molecule sub-batches of it match the oracle (oracle/dmpnn_ref.py) at the fp32
  contract.  A compat batch is not shard-decomposable, so parity is per sub-batch.
"""
import pytest
import torch
import torch.nn as nn

from helpers import FP32_NORM_TOL, assert_parity
from oracle import dmpnn_ref

pytestmark = pytest.mark.gpu

DEV = "cuda"
H = 300


@pytest.fixture(scope="module")
def shard0():
    from notorch_amd.data.synth import make_qm9_batch_vectorized
    from notorch_amd.shard import edge_balanced_ranges

    full = make_qm9_batch_vectorized(1_000_000, seed=1000)
    ranges = edge_balanced_ranges(2 * full.n_bonds, 8)
    a, b = ranges[0]
    assert 120_000 <= b - a <= 130_000
    return full.subset(a, b)


@pytest.fixture(scope="module")
def model():
    from notorch_amd.nn import ChempropBlock, GraphEmbedding

    torch.manual_seed(0)
    emb = GraphEmbedding(42, 13, H).eval()
    blk = ChempropBlock(hidden_dim=H, depth=3).eval()
    return emb.to(DEV), blk.to(DEV)


def _forward(batch, rev_offset, model):
    from notorch_amd.nn import Sum

    emb, blk = model
    G = batch.collate(rev_offset).to(DEV)
    with torch.no_grad():
        out = blk(emb(G))
        return out, Sum()(out)


def test_config4_shard_fixed_mode_decomposes_bitexact(shard0, model):
    from notorch_amd.shard import edge_balanced_ranges

    whole, r_whole = _forward(shard0, "edges", model)
    assert whole.edge_feats.shape == (shard0.num_edges, H)
    parts = [_forward(shard0.subset(a, b), "edges", model) for a, b in edge_balanced_ranges(2 * shard0.n_bonds, 4)]
    assert torch.equal(whole.edge_feats, torch.cat([p[0].edge_feats for p in parts]))
    assert torch.equal(whole.node_feats, torch.cat([p[0].node_feats for p in parts]))
    assert torch.equal(r_whole, torch.cat([p[1] for p in parts]))


def test_config4_shard_compat_mode_runs_and_samples_match_oracle(shard0, model):
    emb, blk = model
    out1, r1 = _forward(shard0, "nodes", model)
    out2, r2 = _forward(shard0, "nodes", model)
    assert torch.isfinite(r1).all()
    assert torch.equal(out1.edge_feats, out2.edge_feats) and torch.equal(r1, r2)  # deterministic
    Ws, bs = dmpnn_ref.block_params(blk)
    Ws = [w.cpu() for w in Ws]
    bs = [b.cpu() for b in bs]
    tab_v = nn.EmbeddingBag.from_pretrained(emb.node.weight.detach().cpu(), mode="sum")
    tab_e = nn.EmbeddingBag.from_pretrained(emb.edge.weight.detach().cpu(), mode="sum")
    n = shard0.num_graphs
    for start in (0, n // 2, n - 64):
        sub = shard0.subset(start, start + 64)
        G = sub.collate("nodes")
        with torch.no_grad():
            Xv, Xe = tab_v(G.node_feats), tab_e(G.edge_feats)
        ref_n, ref_e = dmpnn_ref.chemprop_block(Xv, Xe, G.edge_index, G.rev_index, Ws, bs)
        ref_r = dmpnn_ref.readout(ref_n, G.batch_node_index, len(G), "sum")
        got, got_r = _forward(sub, "nodes", model)
        assert_parity(got.edge_feats, ref_e, FP32_NORM_TOL, f"edge @ {start}")
        assert_parity(got.node_feats, ref_n, FP32_NORM_TOL, f"node @ {start}")
        assert_parity(got_r, ref_r, FP32_NORM_TOL, f"readout @ {start}")
