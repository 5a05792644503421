"""The embedded encoder (GraphEmbedding -> ChempropBlock -> Sum, the reference model path:
embed.py:20-24, chemprop.py:82-83) at config 2 for rocprofv3: K fused steps (the embedding folded into
nt_dmpnn_init_embed), then K unfused steps (nt_embed_bag kernels, then the block).
Usage: python tools/embed_bench.py [--steps 50] [--mols 4096] [--only fused]"""
import argparse
import copy
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--mols", type=int, default=4096)
    p.add_argument("--only", default="fused,unfused")
    a = p.parse_args()
    from notorch_amd.data.synth import make_batch
    from notorch_amd.nn import ChempropBlock, EmbeddedChempropBlock, GraphEmbedding, Sum

    dev = torch.device("cuda")
    torch.manual_seed(0)
    emb = GraphEmbedding(42, 13, 300).to(dev)
    blk = ChempropBlock(hidden_dim=300, depth=3).eval().to(dev)
    G = make_batch("qm9", a.mols, seed=1000).collate("nodes")
    Gd = copy.copy(G).to(dev)
    ro = Sum()
    for mode in a.only.split(","):
        enc = EmbeddedChempropBlock(emb, blk, fuse=mode == "fused").eval()
        with torch.no_grad():
            for _ in range(10):
                ro(enc(Gd))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                ro(enc(Gd))
            torch.cuda.synchronize()
            t = (time.perf_counter() - t0) / a.steps
        print(f"{mode}: {t * 1e3:.4f} ms per step (E={G.num_edges}, V={G.num_nodes})", flush=True)


if __name__ == "__main__":
    main()
