"""Write-bandwidth probe: fill / copy / row-permuted copy of qm9-4096-sized fp32 tensors (torch kernels),
to compare the store rate the fk epilogue reaches with what plain streaming stores reach on the box."""
import statistics

import torch


def t(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
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
    E, h = 77840, 300
    X = torch.randn(E, h, device="cuda")
    Y = torch.empty_like(X)
    big = torch.empty(256 * 1024 * 1024, device="cuda")
    perm = torch.randperm(E, device="cuda")
    local = (torch.arange(E, device="cuda") // 128 * 128 + torch.randperm(128, device="cuda").repeat(E // 128 + 1)[:E]).clamp_(max=E - 1)
    nb = X.numel() * 4
    for name, fn, rd, wr in (
        ("fill 93MB", lambda: Y.fill_(1.0), 0, nb),
        ("fill 1GB", lambda: big.fill_(1.0), 0, big.numel() * 4),
        ("copy 93MB", lambda: Y.copy_(X), nb, nb),
        ("scatter rows random", lambda: Y.index_copy_(0, perm, X), nb, nb),
        ("scatter rows within 128", lambda: Y.index_copy_(0, local, X), nb, nb),
    ):
        us = t(fn)
        print(f"{name:26s} {us:8.1f} us  write {wr / us / 1e3:7.0f} GB/s  total {(rd + wr) / us / 1e3:7.0f} GB/s")


if __name__ == "__main__":
    main()
