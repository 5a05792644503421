"""Micro-benchmark of the individual kernels (device time via torch.cuda events, interleaved
rounds in one process).  Usage: python tools/kbench.py [--mols 4096] [--h 300]"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from notorch_amd import kernels as K  # noqa: E402
from notorch_amd.data.synth import make_batch  # noqa: E402


def timeit(fn, reps=20):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts), min(ts)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mols", type=int, default=4096)
    p.add_argument("--kind", default="qm9")
    p.add_argument("--h", type=int, default=300)
    p.add_argument("--only", default="", help="comma list of kernels to time")
    p.add_argument("--rounds", type=int, default=5)
    a = p.parse_args()
    G = make_batch(a.kind, a.mols, seed=0).collate("nodes").to("cuda")
    V, E, h = G.num_nodes, G.num_edges, a.h
    lay = G._nt_layout
    H = torch.randn(E, h, device="cuda")
    S = torch.randn(V, h, device="cuda")
    Xv = torch.randn(V, h, device="cuda")
    W = torch.randn(h, h, device="cuda") / 17
    b = torch.randn(h, device="cuda")
    Wp = K.pack_weights(W)
    src, rev = G.edge_index[0].contiguous(), G.rev_index
    out = torch.empty_like(H)
    relu = K.act_code(torch.nn.ReLU())
    def upd(variant, cfg="a", mode="0"):
        def f():
            os.environ["NT_UPDATE_KERNEL"] = variant
            os.environ["NT_X6_CFG"] = cfg
            os.environ["NT_PC_MODE"] = mode
            K.dmpnn_update(H, S, src, rev, Wp, b, act=relu, out=out)
        return f

    fns = {
        "update": upd("pc"),
        "pc_noW": upd("pc", mode="2"),
        "pc_oneW": upd("pc", mode="4"),
        "pc_noW_oneW": upd("pc", mode="6"),
        "pc_noMFMA": upd("pc", mode="8"),
        "pc_noW_noMFMA": upd("pc", mode="10"),
        "update_x6": upd("x6"),
        "update_x6b": upd("x6", "b"),
        "update_x6c": upd("x6", "c"),
        "update_x6d": upd("x6", "d"),
        "update_resacc": upd("x6", "r"),
        "abl_noW": upd("x6", "1"),
        "abl_noSH": upd("x6", "2"),
        "abl_noDMA": upd("x6", "3"),
        "abl_noMFMA": upd("x6", "4"),
        "abl_none": upd("x6", "7"),
        "update_glds": upd("glds"),
        "update_ring": upd("ring"),
        "update_stream": upd("stream"),
        "update_tile": upd("tile"),
        "aggregate": lambda: K.segment_reduce(H, lay.dst_ptr, lay.dst_perm, V, act=relu, out=S),
        "init_fused": lambda: K.dmpnn_init(Xv, H, src, lay.dst_ptr, lay.dst_perm, act=relu),
        "node_scatter": lambda: K.segment_reduce(H, lay.dst_ptr, lay.dst_perm, V),
        "pack": lambda: K.pack_weights(W),
    }
    if a.only:
        keep = a.only.split(",")
        fns = {k: v for k, v in fns.items() if k in keep}
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    print(f"V={V} E={E} h={h}")
    res = {n: [] for n in fns}
    for _ in range(a.rounds):  # interleaved rounds
        for name, f in fns.items():
            res[name].append(timeit(f, 10))
    for name, f in fns.items():
        med = statistics.median(r[0] for r in res[name])
        mn = min(r[1] for r in res[name])
        extra = ""
        if name.startswith(("update", "abl", "pc_")):
            extra = f"  {2 * E * h * h / (med * 1e-6) / 1e12:.1f} TF/s"
        else:
            rows = {"aggregate": E + V, "init_fused": 3 * E + V, "node_scatter": E + V, "pack": 0}[name]
            if rows:
                extra = f"  {rows * h * 4 / (med * 1e-6) / 1e9:.0f} GB/s alg"
        print(f"{name:14s} median {med:8.1f} us  min {mn:8.1f} us{extra}")


if __name__ == "__main__":
    main()
