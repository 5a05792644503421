"""Diagnostic: config-2 gradient errors of the kernel backward and of the fp32 CPU oracle, both
against the fp64 oracle autograd, for ReLU (sign-flip prone) and SiLU (smooth)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

import test_gpu_backward as T  # noqa: E402
from helpers import norm_err  # noqa: E402
from notorch_amd.nn import ChempropBlock  # noqa: E402

torch.set_num_threads(16)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
G = T._graph("qm9", n, seed=0)
h = 300
Xv, Xe = T._embed(G, h)
for act, fn in (("ReLU", torch.relu), ("SiLU", torch.nn.functional.silu)):
    torch.manual_seed(1)
    blk = ChempropBlock(h, depth=3, act=T._ACTS[act][0])
    truth = T._oracle_grads(G, Xv, Xe, blk, fn, True, "sum", "sum", torch.float64)
    o32 = T._oracle_grads(G, Xv, Xe, blk, fn, True, "sum", "sum", torch.float32)
    got = T._device_grads(G, Xv, Xe, blk, "sum")
    names = ["dXv", "dXe"] + [f"dW{l}" for l in range(3)] + [f"db{l}" for l in range(3)]
    gl = [got[1], got[2], *got[3], *got[4]]
    ol = [o32[1], o32[2], *o32[3], *o32[4]]
    tl = [truth[1], truth[2], *truth[3], *truth[4]]
    for nm, a, c, b in zip(names, gl, ol, tl):
        print(f"{act:5s} {nm:4s} gpu: max {norm_err(a, b):.2e} l2 {T._rel_l2(a, b):.2e} | "
              f"cpu32: max {norm_err(c, b):.2e} l2 {T._rel_l2(c, b):.2e}", flush=True)
