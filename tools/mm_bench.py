import torch, time, sys
sys.path.insert(0, ".")
from notorch_amd import kernels as K
E, h = 77840, 300
G = torch.randn(E, h, device="cuda"); W = torch.randn(h, h, device="cuda")
Wp = K.pack_weights(W.t().contiguous())
def t(f, n=50):
    for _ in range(5): f()
    torch.cuda.synchronize(); a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n): f()
    b.record(); torch.cuda.synchronize(); return a.elapsed_time(b) / n * 1e3
print("torch.mm us", t(lambda: torch.mm(G, W)))
print("dense_matmul us", t(lambda: K.dense_matmul(G, Wp)))
print("pack W^T us", t(lambda: K.pack_weights(W.t().contiguous())))
