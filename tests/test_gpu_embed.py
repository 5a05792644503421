"""GPU parity of GraphEmbedding on the device and its fusion into the initial gather (SURVEY §8(f)
row 2): nt_embed_bag against nn.EmbeddingBag (embed.py:21-29) on the CPU, nt_dmpnn_init_embed and
EmbeddedChempropBlock bit-identical to the unfused kernels, and the whole embedded encoder against
the CPU oracle (fp32 contract, normalised max error <= 1e-5)."""
import pytest
import torch
import torch.nn as nn

from helpers import assert_parity
from oracle import dmpnn_ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _graph(kind="qm9", n=32, seed=0, rev_offset="nodes"):
    from notorch_amd.data.synth import make_batch

    return make_batch(kind, n, seed=seed).collate(rev_offset)


@pytest.mark.parametrize("h", [300, 13])
def test_embed_bag_matches_embeddingbag(h):
    from notorch_amd import kernels as K

    G = _graph("qm9", 64, seed=1)
    torch.manual_seed(0)
    bag = nn.EmbeddingBag(42, h, mode="sum")
    with torch.no_grad():
        ref = bag(G.node_feats)
        got = K.embed_bag(bag.weight.to(DEV), G.node_feats.to(DEV))
    assert_parity(got, ref, 1e-6, "embed_bag")
    # 7 adds of table rows per bag in ascending column order, from 0: exactly the restated sum
    seq = torch.zeros_like(ref)
    for j in range(G.node_feats.shape[1]):
        seq = seq + bag.weight.detach()[G.node_feats[:, j]]
    assert torch.equal(got.cpu(), seq)


def test_embed_bag_out_of_range_raises():
    from notorch_amd import kernels as K

    T = torch.zeros(5, 8, device=DEV)
    with pytest.raises(IndexError):
        K.embed_bag(T, torch.tensor([[0, 5]], device=DEV))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("h,n", [(256, 48), (300, 48), (13, 48), (512, 48), (300, 3000), (512, 1500)])
def test_init_embed_bit_identical_to_unfused(dtype, h, n):
    """Fused embedding init == embed_bag + nt_dmpnn_init, bit for bit: tables staged in LDS (fp32
    h <= 327, bf16 h <= 655), read from L2 otherwise (fp32 h = 512), scalar pieces (h = 13)."""
    from notorch_amd import kernels as K

    G = _graph("zinc", n, seed=2)
    torch.manual_seed(1)
    Tv = torch.randn(42, h).to(dtype).to(DEV)
    Te = torch.randn(13, h).to(dtype).to(DEV)
    nt, et = G.node_feats.to(DEV), G.edge_feats.to(DEV)
    src, dst = G.edge_index[0].to(DEV), G.edge_index[1].to(DEV)
    seg_ptr, perm = K.csr_build(dst, G.num_nodes)
    Xv, Xe = K.embed_bag(Tv, nt), K.embed_bag(Te, et)
    H0_ref, S_ref = K.dmpnn_init(Xv, Xe, src, seg_ptr, perm)
    H0, S = K.dmpnn_init_embed(Tv, nt, Te, et, src, seg_ptr, perm)
    assert torch.equal(H0, H0_ref) and torch.equal(S, S_ref)
    H0b, none = K.dmpnn_init_embed(Tv, nt, Te, et, src)
    assert none is None and torch.equal(H0b, H0_ref)
    relu = K.act_code(torch.nn.ReLU())
    for reduce in ("mean", "max"):
        H0_ref, S_ref = K.dmpnn_init(Xv, Xe, src, seg_ptr, perm, act=relu, reduce=reduce)
        H0, S = K.dmpnn_init_embed(Tv, nt, Te, et, src, seg_ptr, perm, act=relu, reduce=reduce)
        assert torch.equal(H0, H0_ref) and torch.equal(S, S_ref), reduce


@pytest.mark.parametrize("h", [300, 132])
def test_init_embed_padded_rows_bit_identical(h):
    """ABI 7 ld_out of nt_dmpnn_init_embed: H0 and S on padded rows hold the dense values bit for
    bit (LDS-staged tables at both sizes), the amax chain too."""
    from notorch_amd import kernels as K

    G = _graph("qm9", 400, seed=5)
    torch.manual_seed(2)
    Tv, Te = torch.randn(42, h, device=DEV), torch.randn(13, h, device=DEV)
    nt, et = G.node_feats.to(DEV), G.edge_feats.to(DEV)
    src, dst = G.edge_index[0].to(DEV), G.edge_index[1].to(DEV)
    seg_ptr, perm = K.csr_build(dst, G.num_nodes)
    am0, am1 = torch.zeros(2, device=DEV), torch.zeros(2, device=DEV)
    H0, S = K.dmpnn_init_embed(Tv, nt, Te, et, src, seg_ptr, perm, amax=am0)
    pitch = (h + 7) // 8 * 8 + 8
    H0p, Sp = K.dmpnn_init_embed(Tv, nt, Te, et, src, seg_ptr, perm, amax=am1, pitch=pitch)
    assert H0p.stride(0) == pitch and Sp.stride(0) == pitch
    assert torch.equal(H0p, H0) and torch.equal(Sp, S) and torch.equal(am0, am1)


@pytest.mark.parametrize("h,n,kind", [(300, 4096, "qm9"), (300, 37, "qm9"), (64, 500, "zinc"), (512, 64, "qm9"),
                                      (4, 40, "qm9")])
def test_init_embed_records_bit_identical(h, n, kind):
    """The wave-per-node init over the type records (ABI 8 nt_embed_edge_records) gives the bits of the
    thread-per-piece init: every reduce, relu / identity, padded rows, the amax chain; an out-of-range
    type index contributes a zero row in both."""
    from notorch_amd import kernels as K

    G = _graph(kind, n, seed=9)
    torch.manual_seed(4)
    Tv, Te = torch.randn(42, h, device=DEV), torch.randn(13, h, device=DEV)
    nt, et = G.node_feats.to(DEV), G.edge_feats.to(DEV)
    src, dst = G.edge_index[0].to(DEV), G.edge_index[1].to(DEV)
    seg_ptr, perm = K.csr_build(dst, G.num_nodes)
    rec = K.embed_edge_records(nt, 42, et, 13, src, perm)
    assert rec.shape == (G.num_edges, 4) and torch.equal(rec[:, 0].long(), perm.long())
    if (42 + 13 + 2) * h * 4 > 72 * 1024:  # the tables do not fit the wave init's LDS: refused
        with pytest.raises(RuntimeError, match="records"):
            K.dmpnn_init_embed(Tv, nt, Te, et, src, seg_ptr, perm, records=rec)
        return
    relu = K.act_code(torch.nn.ReLU())
    ident = K.act_code(torch.nn.Identity())
    pitch = (h + 7) // 8 * 8 if h % 8 else h + 8
    for act in (relu, ident):
        for reduce in ("sum", "mean", "max", "min"):
            for ld in (None, pitch):
                am0, am1 = torch.zeros(2, device=DEV), torch.zeros(2, device=DEV)
                H0, S = K.dmpnn_init_embed(Tv, nt, Te, et, src, seg_ptr, perm, act=act, reduce=reduce, amax=am0,
                                           pitch=ld)
                H0r, Sr = K.dmpnn_init_embed(Tv, nt, Te, et, src, seg_ptr, perm, act=act, reduce=reduce, amax=am1,
                                             pitch=ld, records=rec)
                assert torch.equal(H0r, H0) and torch.equal(Sr, S) and torch.equal(am1, am0), (act, reduce, ld)
    # out-of-range indices (validate=False): both paths add a zero row for them
    bad = nt.clone()
    bad[::7, 3] = 99
    rec_bad = K.embed_edge_records(bad, 42, et, 13, src, perm)
    H0, S = K.dmpnn_init_embed(Tv, bad, Te, et, src, seg_ptr, perm, validate=False)
    H0r, Sr = K.dmpnn_init_embed(Tv, bad, Te, et, src, seg_ptr, perm, validate=False, records=rec_bad)
    assert torch.equal(H0r, H0) and torch.equal(Sr, S)


def _modules(h, depth, dtype=torch.float32, **opts):
    from notorch_amd.nn import ChempropBlock, EmbeddedChempropBlock, GraphEmbedding

    torch.manual_seed(3)
    emb = GraphEmbedding(42, 13, h)
    blk = ChempropBlock(hidden_dim=h, depth=depth, **opts)
    return emb, blk, EmbeddedChempropBlock(emb, blk).eval().to(dtype)


@pytest.mark.parametrize("opts", [dict(), dict(reduce="mean", residual=False), dict(depth=0)])
def test_embedded_block_bit_identical_and_oracle(opts):
    opts = dict(opts)
    depth = opts.pop("depth", 3)
    G = _graph("qm9", 128, seed=4)
    emb, blk, fused = _modules(300, depth, **opts)
    with torch.no_grad():
        Xv, Xe = emb(G).node_feats, emb(G).edge_feats  # CPU reference embedding
    Ws, bs = dmpnn_ref.block_params(blk)
    ref_node, ref_edge = dmpnn_ref.chemprop_block(
        Xv, Xe, G.edge_index, G.rev_index, Ws, bs, residual=opts.get("residual", True),
        reduce=opts.get("reduce", "sum"))
    fused = fused.to(DEV)
    Gd = G.to(DEV)
    with torch.no_grad():
        out = fused(Gd)
        unfused = blk(emb(Gd))
    assert torch.equal(out.node_feats, unfused.node_feats)
    assert torch.equal(out.edge_feats, unfused.edge_feats)
    assert_parity(out.node_feats, ref_node, 1e-5, "node")
    assert_parity(out.edge_feats, ref_edge, 1e-5, "edge")


def test_embedded_block_bf16():
    G = _graph("zinc", 64, seed=5)
    emb, blk, fused = _modules(128, 3, torch.bfloat16)
    fused = fused.to(DEV)
    Gd = G.to(DEV)
    with torch.no_grad():
        out = fused(Gd)
        unfused = blk(emb(Gd))
    assert out.edge_feats.dtype == torch.bfloat16
    assert torch.equal(out.node_feats, unfused.node_feats)
    assert torch.equal(out.edge_feats, unfused.edge_feats)


def test_embedded_block_training_falls_back_and_trains_tables():
    G = _graph("qm9", 16, seed=6)
    emb, blk, fused = _modules(32, 2)
    fused = fused.to(DEV).train()
    out = fused(G.to(DEV))
    out.node_feats.pow(2).sum().backward()
    assert emb.node.weight.grad is not None and emb.node.weight.grad.abs().sum() > 0
    assert blk._chemprop_layers()[0].linear.weight.grad is not None


def test_embedded_block_validates_types_once():
    G = _graph("qm9", 8, seed=7)
    _, _, fused = _modules(16, 1)
    fused = fused.to(DEV)
    Gd = G.to(DEV)
    with torch.no_grad():
        fused(Gd)
        bad = Gd.update(node_feats=Gd.node_feats.clone())
        bad.node_feats[0, 0] = 42
        with pytest.raises(IndexError):
            fused(bad)
