"""Training-step timing of ChempropBlock + Sum readout at config 2 (or config 3 with --kind zinc
--h 512 --depth 5 --dtype bf16), as the reference trains: zero_grad, forward, backward and an
Adam(lr=1e-4) step (notorch/lightning_models/model.py:153 optim_factory, :224-241 training_step,
:273 configure_optimizers; Lightning calls optimizer.step() every batch).  The step after the
optimizer sees new weights, so the forward re-packs them (one pack per layer weight).

Modes: `kernel` (the kernel backward, the weight grad per NT_WGRAD) and `torch` (the
recompute-in-torch backward, NT_BWD=torch).  bench.py's `training` key runs this in fresh processes
with --json (the default weight-grad path as the headline, NT_WGRAD=library as a comparison).
Usage: python tools/train_bench.py [--kind qm9] [--mols 4096] [--h 300] [--depth 3] [--dtype f32|bf16]
                                  [--steps 30] [--warmup 10] [--warmup-s 0] [--modes kernel,torch]
                                  [--optim adam|none] [--json]"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from notorch_amd.data.synth import make_batch  # noqa: E402
from notorch_amd.nn import ChempropBlock, Sum  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--kind", default="qm9")
    p.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    p.add_argument("--mols", type=int, default=4096)
    p.add_argument("--seed", type=int, default=1000, help="batch seed (bench.py rank 0: 1000)")
    p.add_argument("--h", type=int, default=300)
    p.add_argument("--depth", type=int, default=3)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--warmup-s", type=float, default=0.0,
                   help="after the counted warm-ups, keep warming up until this many seconds have passed "
                        "(lets the clocks settle in a fresh process)")
    p.add_argument("--modes", default="kernel,torch")
    p.add_argument("--optim", default="adam", choices=["adam", "adam-fused", "none"],
                   help="adam: Adam(lr=1e-4).step() in every training step (the reference's default "
                        "optim_factory; torch's foreach implementation); adam-fused: the same optimizer "
                        "with torch's fused=True implementation; none: forward + backward only")
    p.add_argument("--json", action="store_true", help="print one JSON object instead of the table")
    a = p.parse_args()
    from notorch_amd import _lib

    _lib.load()  # fail loudly if the HIP extension is missing
    dt = {"f32": torch.float32, "bf16": torch.bfloat16}[a.dtype]
    G = make_batch(a.kind, a.mols, seed=a.seed).collate("nodes")
    torch.manual_seed(0)
    ev = torch.nn.EmbeddingBag(42, a.h, mode="sum")
    ee = torch.nn.EmbeddingBag(13, a.h, mode="sum")
    with torch.no_grad():
        Xv, Xe = ev(G.node_feats).to(dt), ee(G.edge_feats).to(dt)
    Gd = G.update(node_feats=Xv, edge_feats=Xe).to("cuda")
    blk = ChempropBlock(a.h, depth=a.depth).to("cuda", dt).train()
    ro = Sum()
    Xv_d = Gd.node_feats.requires_grad_(True)
    Xe_d = Gd.edge_feats.requires_grad_(True)
    E = G.num_edges
    opt = None
    if a.optim != "none":
        opt = torch.optim.Adam(blk.parameters(), lr=1e-4, **({"fused": True} if a.optim == "adam-fused" else {}))

    def step():
        blk.zero_grad(set_to_none=True)
        Xv_d.grad = Xe_d.grad = None
        out = blk(Gd.update(node_feats=Xv_d, edge_feats=Xe_d))
        ro(out).float().pow(2).sum().backward()
        if opt is not None:
            opt.step()

    def fwd():
        with torch.no_grad():
            ro(blk(Gd))

    res = {}
    for mode in a.modes.split(","):
        os.environ["NT_BWD"] = mode
        for name, fn in (("fwd", fwd), (f"train[{mode}]", step)):
            for _ in range(a.warmup):
                fn()
            torch.cuda.synchronize()
            t_end = time.perf_counter() + a.warmup_s
            while time.perf_counter() < t_end:
                fn()
                torch.cuda.synchronize()
            # back-to-back steps as a training loop runs them (no host sync between steps, so the
            # host's autograd / optimizer bookkeeping overlaps the device work of the previous step):
            # rounds of `chunk` steps between two events, the median round per step
            ts = []
            chunk = max(1, min(10, a.steps))
            for _ in range(max(1, a.steps // chunk)):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(chunk):
                    fn()
                e.record()
                e.synchronize()
                ts.append(s.elapsed_time(e) / chunk)
            res[name] = statistics.median(ts)
    if a.json:
        print(json.dumps({
            "V": G.num_nodes, "E": E, "h": a.h, "depth": a.depth, "dtype": a.dtype,
            "weight_grad": os.environ.get("NT_WGRAD", "default"), "optim": a.optim,
            "warmup": a.warmup, "steps": a.steps,
            "ms": res, "edge_messages_per_s": {k: E * a.depth / (v * 1e-3) for k, v in res.items()},
        }), flush=True)
        return
    print(f"{a.kind} V={G.num_nodes} E={E} h={a.h} depth={a.depth} {a.dtype} optim={a.optim}")
    for k, v in res.items():
        print(f"{k:14s} {v:8.3f} ms/step  {E * a.depth / (v * 1e-3):.3e} edge-msg/s")


if __name__ == "__main__":
    main()
