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

    deg = (lay.dst_ptr[1:] - lay.dst_ptr[:-1]).max().item()
    plan = K.tile_plan(lay.dst_ptr, E, int(deg))
    S2 = torch.empty_like(S)

    ident = torch.arange(E, dtype=torch.int32, device="cuda")
    fake_d = (ident.long() * V // E).to(torch.int32)  # monotone, < V: timing stand-in only
    eplan = (torch.arange(0, E + 64, 64, dtype=torch.int32, device="cuda").clamp_(max=E), (E + 63) // 64, fake_d)

    def fused_edge_order():
        os.environ["NT_PS_ABL"] = "0"
        K.dmpnn_update_fused(H, S, src, rev, Wp, b, act=relu, plan=eplan, perm=ident, agg_act=relu,
                             out=out, S_out=S2)

    def fused(kmid=None, with_plan=True, abl=0, kern="pk", pkabl=0):
        def f():
            os.environ["NT_FUSED_KERNEL"] = kern
            os.environ["NT_PS_ABL"] = str(abl)
            os.environ["NT_PK_ABL"] = str(pkabl)
            if kmid is not None:
                os.environ["NT_PS_KMID"] = str(kmid)
            else:
                os.environ.pop("NT_PS_KMID", None)
            K.dmpnn_update_fused(H, S, src, rev, Wp, b, act=relu, plan=plan if with_plan else None,
                                 perm=lay.dst_perm, agg_act=relu, out=out,
                                 S_out=S2 if with_plan else None)
        return f

    fns = {
        "fused": fused(),
        "fused_ps": fused(kern="ps"),
        "pk_unfused": fused(with_plan=False),
        "pk_noprod": fused(pkabl=1),
        "pk_noprod_noW": fused(pkabl=3),
        "pk_noprod_nores": fused(pkabl=5),
        "pk_noprod_noW_nores": fused(pkabl=7),
        "pk_noprod_nomfma": fused(pkabl=9),
        "pk_noprod_all": fused(pkabl=15),
        "fused_edgeorder": fused_edge_order,
        "fused_k0": fused(0, kern="ps"),
        "fused_k3": fused(3, kern="ps"),
        "fused_k7": fused(7, kern="ps"),
        "ps": fused(with_plan=False, kern="ps"),
        "ps_noprod": fused(with_plan=False, abl=1, kern="ps"),
        "ps_nomfma": fused(with_plan=False, abl=2, kern="ps"),
        "ps_noW": fused(with_plan=False, abl=4, kern="ps"),
        "ps_nosplit": fused(with_plan=False, abl=8, kern="ps"),
        "ps_noprod_noW": fused(with_plan=False, abl=5, kern="ps"),
        "ps_noprod_nosplit": fused(with_plan=False, abl=9, kern="ps"),
        "ps_noprod_noW_nosplit": fused(with_plan=False, abl=13, kern="ps"),
        "ps_noprod_nomfma": fused(with_plan=False, abl=3, kern="ps"),
        "ps_nomfma_noW": fused(with_plan=False, abl=6, kern="ps"),
        "fused_noprod": fused(abl=1, kern="ps"),
        "fused_noHres": fused(abl=32, kern="ps"),
        "fused_nostore": fused(abl=64, kern="ps"),
        "fused_noHres_nostore": fused(abl=96, kern="ps"),
        "fused_nomfma_noHres": fused(abl=34, kern="ps"),
        "fused_nomfma_noHres_nostore": fused(abl=98, kern="ps"),
        "fused_nomfma": fused(abl=2, kern="ps"),
        "update": upd("as"),
        "update_pc": upd("pc"),
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
        if name.startswith(("update", "abl", "pc_", "fused", "ps", "pk")):
            extra = f"  {2 * E * h * h / (med * 1e-6) / 1e12:.1f} TF/s"
        else:
            rows = {"aggregate": E + V, "init_fused": 3 * E + V, "node_scatter": E + V, "pack": 0}[name]
            if rows:
                extra = f"  {rows * h * 4 / (med * 1e-6) / 1e9:.0f} GB/s alg"
        print(f"{name:14s} median {med:8.1f} us  min {mn:8.1f} us{extra}")


if __name__ == "__main__":
    main()
