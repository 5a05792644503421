"""A/B of the fp32 fused layer walks on one batch: update_fk_kernel (nt_debug_set_fw(0)) against
update_fw_kernel (nt_debug_set_fw(1)) on the same 128-row plan -- bit-exact comparison of H_out,
S_out and the amax chain, then interleaved timings.
Usage: python tools/fw_check.py [--kind qm9] [--mols 4096] [--h 300] [--rev nodes] [--rounds 5]"""
import argparse
import ctypes
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from notorch_amd import _lib  # noqa: E402
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
    p.add_argument("--kind", default="qm9")
    p.add_argument("--mols", type=int, default=4096)
    p.add_argument("--h", type=int, default=300)
    p.add_argument("--rev", default="nodes")
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--rows", type=int, default=128)
    p.add_argument("--agg", default="relu")
    p.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    a = p.parse_args()
    lib = _lib.load()
    setfw = getattr(lib, "nt_debug_set_fw")
    setfw.argtypes = [ctypes.c_int]
    G = make_batch(a.kind, a.mols, seed=0).collate(a.rev).to("cuda")
    V, E, h = G.num_nodes, G.num_edges, a.h
    lay = G._nt_layout
    gen = torch.Generator(device="cuda").manual_seed(0)
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    H = torch.randn(E, h, device="cuda", generator=gen).to(dt)
    S = torch.randn(V, h, device="cuda", generator=gen).to(dt)
    W = (torch.randn(h, h, device="cuda", generator=gen) / 17).to(dt)
    b = torch.randn(h, device="cuda", generator=gen).to(dt)
    Wp = K.pack_weights(W)
    src, rev = G.edge_index[0].contiguous(), G.rev_index
    relu = K.act_code(torch.nn.ReLU())
    agg = relu if a.agg == "relu" else K.act_code(torch.nn.Identity())
    amax = None
    if dt == torch.float32:
        amax = torch.zeros(2, device="cuda")
        K.absmax(H, amax[0:1])
        K.absmax(S, amax[1:2])
    deg = int((lay.dst_ptr[1:] - lay.dst_ptr[:-1]).max().item())
    plan = K.tile_plan(lay.dst_ptr, E, deg, rows=a.rows, ncu=K.PLAN_NCU)
    rt = K.dmpnn_row_table(lay.dst_perm, plan[2], src, rev, V)
    plan64 = K.tile_plan(lay.dst_ptr, E, deg, rows=64, ncu=K.PLAN_NCU)
    rt64 = K.dmpnn_row_table(lay.dst_perm, plan64[2], src, rev, V)
    outs = {}

    def run(v, out, S2, am):
        # bf16: the default bf16 kernel takes 64-row plans only, so v = 0 is the 64-row walk too
        pl, rtab, rows = (plan64, rt64, 64) if (v == 2 or (v == 0 and dt != torch.float32)) else (plan, rt, a.rows)

        def f():
            setfw(1 if v == 1 else 0)
            K.dmpnn_update_fused(H, S, src, rev, Wp, b, act=relu, plan=pl, tile_rows=rows, max_in_degree=deg,
                                 perm=lay.dst_perm, agg_act=agg, amax_in=amax, amax_out=am, row_table=rtab, out=out,
                                 S_out=S2)
        return f

    fns = {}
    for v in (0, 1, 2):
        out, S2 = torch.full_like(H, float("nan")), torch.full_like(S, float("nan"))
        am = torch.zeros(2, device="cuda") if dt == torch.float32 else None
        outs[v] = (out, S2, am)
        fns[v] = run(v, out, S2, am)
        fns[v]()
    torch.cuda.synchronize()
    st = K.device_status() if hasattr(K, "device_status") else None
    print(f"{a.kind}-{a.mols} rev={a.rev} V={V} E={E} h={h} deg={deg} tiles={plan[1]} status={st}")
    (o0, s0, m0), (o1, s1, m1) = outs[0], outs[1]
    eqH, eqS = torch.equal(o0, o1), torch.equal(s0, s1)
    eqM = m0 is None or torch.equal(m0, m1)
    o0, o1, s0, s1 = o0.float(), o1.float(), s0.float(), s1.float()
    dH = (o0 - o1).abs().max().item() / o0.abs().max().item()
    dS = (s0 - s1).abs().max().item() / s0.abs().max().item()
    print(f"bit-exact H {eqH} S {eqS} amax {eqM}  (norm max diff H {dH:.3e} S {dS:.3e}; nan {o1.isnan().sum().item()})")
    if not eqH:  # where the walks disagree: rows by position in their tile, columns by tile / wave
        diff = (o0 != o1)
        nd = int(diff.sum())
        rows = diff.any(1).nonzero().flatten()
        cols = diff.any(0).nonzero().flatten()
        tp = plan[0].cpu().long()
        dsts_pos = torch.empty(E, dtype=torch.long)
        dsts_pos[lay.dst_perm.cpu().long()] = torch.arange(E)
        pos = dsts_pos[rows.cpu()]
        tile = torch.searchsorted(tp, pos, right=True) - 1
        inrow = pos - tp[tile]
        print(f"  H mismatches: {nd} elements in {rows.numel()} rows, {cols.numel()} columns")
        print(f"  row-in-tile histogram (by 16): {torch.bincount(inrow // 16, minlength=8).tolist()}")
        ct = cols.cpu() // 16
        print(f"  column tiles: {torch.bincount(ct, minlength=(h + 15) // 16).tolist()}")
        print(f"  tiles touched: {tile.unique().numel()} of {plan[1]}; first rows {rows[:8].tolist()} cols {cols[:8].tolist()}")
        r0 = rows[0].item()
        c0 = diff[r0].nonzero().flatten()[:4].tolist()
        print(f"  row {r0}: fk {o0[r0, c0].tolist()} fw {o1[r0, c0].tolist()}")
    o2, s2, m2 = outs[2]
    print(f"fk 64-row walk bit-exact vs 128-row: H {torch.equal(o0, o2.float())} S {torch.equal(s0, s2.float())}; "
          f"fw vs 64-row: H {torch.equal(o1, o2.float())} S {torch.equal(s1, s2.float())} "
          f"(norm max diff H {(o1 - o2.float()).abs().max().item() / o2.float().abs().max().item():.3e})")
    res = {0: [], 1: [], 2: []}
    for _ in range(a.rounds):
        for v in (0, 1, 2):
            res[v].append(timeit(fns[v]))
    for v, name in ((0, "fk128"), (1, "fw128"), (2, "fk64")):
        med = statistics.median(res[v])
        print(f"{name}: median {med:7.1f} us  {2 * E * h * h / (med * 1e-6) / 1e12:6.1f} TF/s fp32-equivalent")
    if hasattr(lib, "nt_debug_fw_stamps"):  # FW_STAMP build: where the fw walk's cycles go
        import ctypes as C
        buf = (C.c_ulonglong * 6)()
        lib.nt_debug_fw_stamps(buf)  # reset
        for _ in range(10):
            fns[1]()
        torch.cuda.synchronize()
        lib.nt_debug_fw_stamps(buf)
        k, e, f, t, w, tot = list(buf)
        print(f"stamps per wave per launch: K loops {k / w:.0f} cyc ({k / t:.0f} per tile), epilogues {e / w:.0f} "
              f"({e / t:.0f} per tile), first step pair {f / t:.0f} per tile, whole walk {tot / w:.0f}; "
              f"tiles/wave {t / w * 10 / 10:.2f}")
    setfw(-1)
    if not (eqH and eqS and eqM):
        sys.exit(3)


if __name__ == "__main__":
    main()
