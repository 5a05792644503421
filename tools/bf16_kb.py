"""Device time of the bf16 fused layer kernel (config 3 shape: zinc-4096, h = 512) for the library
selected by NT_LIB (A/B and ablation variants, tools/r5_bf16_abl.sh).
Usage: python tools/bf16_kb.py [--kind zinc] [--mols 4096] [--h 512] [--rounds 5]"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from notorch_amd import kernels as K  # noqa: E402
from notorch_amd.data.synth import make_batch  # noqa: E402


def timeit(fn, reps=10):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--kind", default="zinc")
    p.add_argument("--mols", type=int, default=4096)
    p.add_argument("--h", type=int, default=512)
    p.add_argument("--rounds", type=int, default=5)
    a = p.parse_args()
    G = make_batch(a.kind, a.mols, seed=0).collate("nodes").to("cuda")
    V, E, h = G.num_nodes, G.num_edges, a.h
    lay = G._nt_layout
    gen = torch.Generator(device="cuda").manual_seed(0)
    bf = torch.bfloat16
    H = torch.randn(E, h, device="cuda", generator=gen).to(bf)
    S = torch.randn(V, h, device="cuda", generator=gen).to(bf)
    W = (torch.randn(h, h, device="cuda", generator=gen) / 23).to(bf)
    b = torch.randn(h, device="cuda", generator=gen).to(bf)
    Wp = K.pack_weights(W)
    src, rev = G.edge_index[0].contiguous(), G.rev_index
    relu = K.act_code(torch.nn.ReLU())
    deg = int((lay.dst_ptr[1:] - lay.dst_ptr[:-1]).max().item())
    rows = K.fused_tile_rows(h, bf) if hasattr(K, "fused_tile_rows") else 64
    plan = K.tile_plan(lay.dst_ptr, E, deg, rows=rows, ncu=K.PLAN_NCU)
    rt = K.dmpnn_row_table(lay.dst_perm, plan[2], src, rev, V)
    out, S2 = torch.empty_like(H), torch.empty_like(S)

    def f():
        K.dmpnn_update_fused(H, S, src, rev, Wp, b, act=relu, plan=plan, tile_rows=rows, max_in_degree=deg,
                             perm=lay.dst_perm, agg_act=relu, row_table=rt, out=out, S_out=S2)
    f()
    torch.cuda.synchronize()
    res = [timeit(f) for _ in range(a.rounds)]
    med = statistics.median(res)
    alg = (4 * E * h * 2 + V * h * 2) / (med * 1e-6) / 1e12
    print(f"{a.kind}-{a.mols} V={V} E={E} h={h} rows={rows}: median {med:7.1f} us  "
          f"(~{alg:.2f} TB/s of H/S/H' rows)  lib={os.environ.get('NT_LIB', '')}")


if __name__ == "__main__":
    main()
