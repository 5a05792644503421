"""Coarse per-phase cycles of the fp32 layer kernel at config 2 from a FK_STAMP variant build
(make VARIANT=<v> EXTRA="-DFK_STAMP=1 ..."; NT_LIB=variant:<v>): per wave and launch, the K-loop
cycles, the epilogue cycles and the first two k-steps of every (tile, chunk) unit."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from notorch_amd import _lib  # noqa: E402
from notorch_amd import kernels as K  # noqa: E402
from notorch_amd.data.synth import make_batch  # noqa: E402


def main():
    lib = _lib.load()
    fn = lib.nt_debug_fk_stamps
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    G = make_batch("qm9", 4096, seed=0).collate("nodes").to("cuda")
    V, E, h = G.num_nodes, G.num_edges, 300
    lay = G._nt_layout
    g = torch.Generator(device="cuda").manual_seed(0)
    H = torch.randn(E, h, device="cuda", generator=g)
    S = torch.randn(V, h, device="cuda", generator=g)
    W = torch.randn(h, h, device="cuda", generator=g) / 17
    b = torch.randn(h, device="cuda", generator=g)
    Wp = K.pack_weights(W)
    src, rev = G.edge_index[0].contiguous(), G.rev_index
    deg = int((lay.dst_ptr[1:] - lay.dst_ptr[:-1]).max().item())
    plan = K.tile_plan(lay.dst_ptr, E, deg, rows=128, ncu=K.PLAN_NCU)
    rt = K.dmpnn_row_table(lay.dst_perm, plan[2], src, rev, V)
    relu = K.act_code(torch.nn.ReLU())
    amax = torch.zeros(2, device="cuda")
    K.absmax(H, amax[0:1])
    K.absmax(S, amax[1:2])
    out, S2 = torch.empty_like(H), torch.empty_like(S)

    def run():
        K.dmpnn_update_fused(H, S, src, rev, Wp, b, act=relu, plan=plan, tile_rows=128, max_in_degree=deg,
                             perm=lay.dst_perm, agg_act=relu, amax_in=amax, row_table=rt, out=out, S_out=S2)

    for _ in range(20):
        run()
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 5)()
    fn(buf)  # reset
    n = 50
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(n):
        run()
    ev[1].record()
    torch.cuda.synchronize()
    fn(buf)
    k, e, f, units, waves = list(buf)
    us = ev[0].elapsed_time(ev[1]) * 1e3 / n
    w = waves / n
    print(f"launch {us:.1f} us; per wave per launch (cycles): K loop {k / waves:.0f}, epilogue {e / waves:.0f}, "
          f"first two k-steps of the units {f / waves:.0f}; units per wave {units / waves:.2f}; waves/launch {w:.0f}")


if __name__ == "__main__":
    main()
