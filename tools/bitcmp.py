"""Bit-identity of two library builds on the block forward: run with NT_LIB=<a>, then with NT_LIB=<b>,
each saving its outputs (--save TAG), then --compare TAG_A TAG_B.  Seeded config-2-shaped batch (and a
smaller one), h=300, depth=3, fp32, both rev modes."""
import argparse
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")


def run(tag):
    from notorch_amd.data.synth import make_batch
    from notorch_amd.nn import ChempropBlock, Sum

    res = {}
    for n, rev in ((4096, "nodes"), (1000, "edges"), (37, "nodes")):
        G = make_batch("qm9", n, seed=7).collate(rev)
        torch.manual_seed(0)
        h = 300
        Xv, Xe = torch.randn(G.num_nodes, h), torch.randn(G.num_edges, h)
        blk = ChempropBlock(hidden_dim=h, depth=3).eval().cuda()
        Gd = G.update(node_feats=Xv, edge_feats=Xe).to("cuda")
        with torch.no_grad():
            out = blk(Gd)
            r = Sum()(out)
        torch.cuda.synchronize()
        res[f"{n}{rev}"] = [digest(t) for t in (out.edge_feats, out.node_feats, r)]
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, f"bitcmp_{tag}.json"), "w") as f:
        json.dump(res, f)
    print(tag, "saved")


def digest(t):
    """(sha256 of the bytes, float64 sum): equal digests = bit-identical tensors"""
    a = t.detach().contiguous().cpu()
    return [hashlib.sha256(a.numpy().tobytes()).hexdigest(), float(a.double().sum())]


def compare(ta, tb):
    A = json.load(open(os.path.join(OUT, f"bitcmp_{ta}.json")))
    B = json.load(open(os.path.join(OUT, f"bitcmp_{tb}.json")))
    ok = True
    for k in A:
        for name, x, y in zip(("edge", "node", "readout"), A[k], B[k]):
            same = x[0] == y[0]
            ok &= same
            print(f"{k:12s} {name:8s} bit-identical={same} sums {x[1]:.9e} / {y[1]:.9e}")
    print("BITCMP", "OK" if ok else "DIFF")
    return 0 if ok else 1


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--save")
    p.add_argument("--compare", nargs=2)
    a = p.parse_args()
    if a.save:
        run(a.save)
    else:
        sys.exit(compare(*a.compare))
