"""Does the in-memory edge order matter for the fused update?  Times the update launches of a
forward on (a) the collated graph (edge order = molecule / bond order; the fused tiles walk it
through dst_perm) and (b) the same graph with its edges renumbered in dst-sorted order (dst_perm =
identity, every tile's rows contiguous in HBM).  Usage: python tools/order_probe.py"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from notorch_amd.data.models.graph import BatchedGraph  # noqa: E402
from notorch_amd.data.synth import make_batch  # noqa: E402
from notorch_amd.nn import ChempropBlock  # noqa: E402
from notorch_amd.nn.gnn import _engine  # noqa: E402


def sorted_copy(G):
    dst = G.edge_index[1]
    perm = torch.argsort(dst, stable=True)
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(perm.numel())
    return BatchedGraph(G.node_feats, G.edge_feats[perm], G.edge_index[:, perm], inv[G.rev_index[perm]],
                        batch_node_index=G.batch_node_index, batch_edge_index=G.batch_edge_index[perm],
                        size=len(G))


def run(kind, n, h, d, dtype):
    G = make_batch(kind, n, seed=0).collate("nodes")
    torch.manual_seed(0)
    G = G.update(node_feats=torch.randn(G.num_nodes, h).to(dtype), edge_feats=torch.randn(G.num_edges, h).to(dtype))
    blk = ChempropBlock(h, depth=d).eval().to(dtype).cuda()
    for name, g in (("collated", G), ("dst-sorted", sorted_copy(G))):
        gd = g.to("cuda")
        with torch.no_grad():
            for _ in range(3):
                blk(gd)
            ev = []
            _engine.UPDATE_EVENTS = ev
            torch.cuda.synchronize()
            for _ in range(10):
                blk(gd)
            torch.cuda.synchronize()
            _engine.UPDATE_EVENTS = None
        t = statistics.mean(a.elapsed_time(b) for a, b in ev) * 1e3
        print(f"{kind}-{n} {dtype} {name:10s}: update {t:7.1f} us/launch")


run("qm9", 4096, 300, 3, torch.float32)
run("zinc", 4096, 512, 5, torch.bfloat16)
