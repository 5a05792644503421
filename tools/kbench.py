"""Micro-benchmark of the individual fp32 forward kernels on one qm9-shaped batch (device time via
torch.cuda events, interleaved rounds in one process).  Also the driver for the per-kernel PMC passes
(tools/pmc_update.sh).  Usage: python tools/kbench.py [--mols 4096] [--h 300] [--only fk_fused,init]"""
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
    p.add_argument("--abl", default="", help="NT_LIB=diag: comma list of NT_FK_ABL ablations of fk_fused")
    a = p.parse_args()
    G = make_batch(a.kind, a.mols, seed=0).collate("nodes").to("cuda")
    V, E, h = G.num_nodes, G.num_edges, a.h
    lay = G._nt_layout
    gen = torch.Generator(device="cuda").manual_seed(0)
    H = torch.randn(E, h, device="cuda", generator=gen)
    S = torch.randn(V, h, device="cuda", generator=gen)
    Xv = torch.randn(V, h, device="cuda", generator=gen)
    W = torch.randn(h, h, device="cuda", generator=gen) / 17
    b = torch.randn(h, device="cuda", generator=gen)
    Wp = K.pack_weights(W)
    src, rev = G.edge_index[0].contiguous(), G.rev_index
    out = torch.empty_like(H)
    H2 = torch.randn(E, h, device="cuda", generator=gen)
    S2 = torch.empty_like(S)
    R = torch.empty(len(G), h, device="cuda")
    relu = K.act_code(torch.nn.ReLU())
    amax = torch.zeros(2, device="cuda")
    K.absmax(H, amax[0:1])
    K.absmax(S, amax[1:2])
    amax_out = torch.zeros(2, device="cuda")
    deg = int((lay.dst_ptr[1:] - lay.dst_ptr[:-1]).max().item())
    plans = {}
    for rows in (64, 128):
        plan = K.tile_plan(lay.dst_ptr, E, deg, rows=rows, ncu=K.PLAN_NCU)
        rt = K.dmpnn_row_table(lay.dst_perm, plan[2], src, rev, V)
        plans[rows] = (plan, rt)

    def fk(rows, abl=None):
        plan, rt = plans[rows]

        def f():
            os.environ["NT_FK_ABL"] = str(abl or 0)
            K.dmpnn_update_fused(H, S, src, rev, Wp, b, act=relu, plan=plan, tile_rows=rows, max_in_degree=deg,
                                 perm=lay.dst_perm, agg_act=relu, amax_in=amax, amax_out=amax_out,
                                 row_table=rt, out=out, S_out=S2)
        return f

    def fk_stagger(n):
        f0 = fk(128)

        def f():
            os.environ["NT_FK_STAGGER"] = str(n)
            try:
                f0()
            finally:
                os.environ["NT_FK_STAGGER"] = "0"
        return f

    def fk_plain():
        K.dmpnn_update_fused(H, S, src, rev, Wp, b, act=relu, amax_in=amax, amax_out=amax_out, out=out)

    fns = {
        "fk_fused": fk(128),
        "fk_fused64": fk(64),
        "fk_plain": fk_plain,
        "fk_stagger1": fk_stagger(1),
        "fk_stagger2": fk_stagger(2),
        "fk_stagger4": fk_stagger(4),
        "init": lambda: K.dmpnn_init(Xv, H, src, lay.dst_ptr, lay.dst_perm, act=relu, amax=amax_out),
        "init_noamax": lambda: K.dmpnn_init(Xv, H, src, lay.dst_ptr, lay.dst_perm, act=relu),
        "fk_noamax": lambda: K.dmpnn_update_fused(H, S, src, rev, Wp, b, act=relu, plan=plans[128][0], tile_rows=128,
                                                  max_in_degree=deg, perm=lay.dst_perm, agg_act=relu, amax_in=amax,
                                                  row_table=plans[128][1], out=out, S_out=S2),
        "init_only": lambda: K.dmpnn_init(Xv, H, src, act=relu, amax=amax_out),
        # bandwidth ceilings of the init's traffic: E-row copy (2 rows / edge), E-row add (3 rows / edge)
        "readout": lambda: K.segment_reduce(S, lay.mol_ptr, None, len(G), out=R),
        "copy": lambda: out.copy_(H),
        "add": lambda: torch.add(H, H2, out=out),
        "absmax": lambda: K.absmax(H, amax_out[0:1]),
        "pack": lambda: K.pack_weights(W),
    }
    for n in filter(None, a.abl.split(",")):
        fns[f"fk_abl{n}"] = fk(64, int(n))
    if a.only:
        keep = a.only.split(",") + [k for k in fns if k.startswith("fk_abl")]
        fns = {k: v for k, v in fns.items() if k in keep}
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    print(f"V={V} E={E} h={h} max_in_degree={deg} tiles128={plans[128][0][1]} tiles64={plans[64][0][1]}")
    res = {n: [] for n in fns}
    for _ in range(a.rounds):  # interleaved rounds
        for name, f in fns.items():
            res[name].append(timeit(f, 10))
    for name in fns:
        med = statistics.median(r[0] for r in res[name])
        mn = min(r[1] for r in res[name])
        extra = ""
        if name.startswith("fk"):
            extra = f"  {2 * E * h * h / (med * 1e-6) / 1e12:.1f} TF/s fp32-equivalent"
        elif name in ("init", "init_noamax", "init_only", "copy", "add", "absmax"):
            rows = {"init": 3 * E + V, "init_noamax": 3 * E + V, "init_only": 3 * E, "copy": 2 * E, "add": 3 * E,
                    "absmax": E}[name]
            extra = f"  {rows * h * 4 / (med * 1e-6) / 1e9:.0f} GB/s alg"
        print(f"{name:12s} median {med:8.1f} us  min {mn:8.1f} us{extra}")


if __name__ == "__main__":
    main()
