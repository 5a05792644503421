"""bench.py — edge-messages/s of the D-MPNN forward (ChempropBlock + Sum readout) on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 launched by
``torch.distributed.run`` (one rank per GPU, RCCL).  Rank 0 prints ONE JSON line.

Workload (BASELINE.json configs[1]): per GPU a 4096-molecule QM9-shaped batch (synthetic, seeded
per rank -> weak scaling), hidden 300, depth 3, fp32, ReLU, residual, sum reduce, reference
collate semantics (rev offset by nodes).  A "step" = one forward of ChempropBlock + Sum readout
with the collated graph (incl. its CSR layout) and the embedded features already resident in HBM.
value = sum over ranks of E_r * depth * K / max over ranks of the timed seconds.

Also reported: ``roofline`` for the dominant kernel (nt_dmpnn_update_fused, or nt_dmpnn_update on
the unfused path; per-launch duration from
torch.cuda events recorded on the launch stream around every launch inside the timed region) and
``cpu_baseline`` (the oracle restatement on the host CPU, rank 0, N=1, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from notorch_amd.shard import aggregate_throughput, dist_env  # noqa: E402

METRIC = "edge-messages/sec D-MPNN depth=3 h=300, QM9-shaped batches, 1/2/4/8 MI355X"
PEAK_FP32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense fp32 MFMA (= vector) peak
PEAK_HBM_GBPS = 8000.0
PEAK_BF16_MFMA_TFLOPS = 2500.0  # dense bf16 MFMA (MI355X_MICROARCH.md)

WORKLOADS = {
    # name: (generator, molecules per GPU, hidden, depth, storage dtype)
    "qm9-4096": ("qm9", 4096, 300, 3, "f32"),  # BASELINE config 2 (the metric's configuration)
    "qm9-32k": ("qm9", 32768, 300, 3, "f32"),  # HBM-scale batch (working set >> Infinity Cache)
    "qm9-125k": ("qm9", 125000, 300, 3, "f32"),  # config 4: one GPU's whole 1M/8 shard in one batch
    "zinc-4096-bf16": ("zinc", 4096, 512, 5, "bf16"),  # BASELINE config 3 (bf16)
    "zinc-4096": ("zinc", 4096, 512, 5, "f32"),  # config 3 shape, fp32
    "polymer-16": ("polymer", 16, 300, 3, "f32"),  # config 5 shape
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--workload", default="qm9-4096", choices=sorted(WORKLOADS))
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-embedded", action="store_true", help="skip the embedded-encoder measurement")
    p.add_argument("--pmc-csv", default=None,
                   help="comma-separated rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE counter CSVs of the "
                   "same command (tools/profile.sh) to fill roofline.traffic")
    return p.parse_args()


def forward_bytes_flops(V, E, B, h, d, b=4):
    """SURVEY §8(d) minimal-traffic model of the fused forward + its MFMA flops."""
    rows = b * h * ((2 * d + 3) * (E + V) + B)
    idx = 4 * ((3 * d + 2) * E + (d + 1) * (V + 1) + (B + 1))
    wts = d * (h * h + h) * b
    return rows + idx + wts, 2 * d * E * h * h


def fused_bytes(V, E, h, b=4):
    """Algorithmic bytes of ONE nt_dmpnn_update_fused launch (SURVEY §8(d) minimal model of a
    layer: read H, read S, write H', write S' = 2E + 2V rows; int32 src/rev/perm; weights once)."""
    return b * h * (2 * E + 2 * V) + 4 * 3 * E + (h * h + h) * b


def update_bytes(V, E, h, b=4):
    """Algorithmic HBM bytes of ONE nt_dmpnn_update launch: read H[e], gather S[src[e]] and
    H[rev[e]], write H_out[e] (4 rows per edge), src+rev int64, weights once."""
    return 4 * E * h * b + 16 * E + (h * h + h) * b


def cpu_baseline(G, Xv, Xe, Ws, bs, depth, budget_s):
    """Oracle restatement (ATen CPU) timed on the host; median of runs within the budget."""
    from oracle import dmpnn_ref

    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    threads = max(1, min(16, cores))
    torch.set_num_threads(threads)
    ei, rev, bni, B = G.edge_index.cpu(), G.rev_index.cpu(), G.batch_node_index.cpu(), len(G)
    Xv, Xe = Xv.cpu(), Xe.cpu()
    Ws = [w.detach().cpu() for w in Ws]
    bs = [b.detach().cpu() for b in bs]

    def one():
        with torch.inference_mode():
            n, _ = dmpnn_ref.chemprop_block(Xv, Xe, ei, rev, Ws, bs)
            dmpnn_ref.readout(n, bni, B, "sum")

    one()  # warm-up
    times, t_start = [], time.perf_counter()
    while (time.perf_counter() - t_start < budget_s and len(times) < 200) or len(times) < 3:
        t0 = time.perf_counter()
        one()
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    E = ei.shape[1]
    return {
        "value": E * depth / med,
        "unit": "edge-messages/s",
        "cores": threads,
        "kind": "port",
        "sample": f"oracle/dmpnn_ref.py (ATen CPU restatement of chemprop.py+agg.py) on the same "
        f"{B}-molecule batch, fp32, torch.set_num_threads({threads}), median of {len(times)} "
        f"forwards ({med * 1e3:.1f} ms each) after 1 warm-up; host cpus visible {cores}",
    }


def read_pmc_traffic(paths, kernel_substr="update"):
    """Average HBM bytes per launch of the update kernel from rocprofv3 --pmc counter_collection
    CSVs (comma-separated; FETCH_SIZE and WRITE_SIZE come from separate passes).
    gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reads 1/2 of wide streaming reads
    -> x2; WRITE_SIZE is exact for 16-B stores.  Both are in KB."""
    import csv

    fetch, write, n_f, n_w = 0.0, 0.0, set(), set()
    for path in paths.split(","):
        with open(path) as f:
            for row in csv.DictReader(f):
                kn = row.get("Kernel_Name", "")
                if kernel_substr not in kn or "pack" in kn:
                    continue
                name, val = row.get("Counter_Name"), float(row.get("Counter_Value", 0))
                did = (path, row.get("Dispatch_Id"))
                if name == "FETCH_SIZE":
                    fetch += val
                    n_f.add(did)
                elif name == "WRITE_SIZE":
                    write += val
                    n_w.add(did)
    if not n_f and not n_w:
        return None
    per = 0.0
    if n_f:
        per += 2.0 * fetch / len(n_f) * 1024
    if n_w:
        per += write / len(n_w) * 1024
    return per


def main():
    args = parse()
    env = dist_env()
    if env.distributed:
        torch.cuda.set_device(env.local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", env.local_rank))
    dev = torch.device("cuda", env.local_rank)

    from notorch_amd import _lib
    from notorch_amd.data.synth import make_batch
    from notorch_amd.nn import ChempropBlock, EmbeddedChempropBlock, GraphEmbedding, Sum
    from notorch_amd.nn.gnn import _engine

    _lib.load()  # fail loudly if the HIP extension is missing
    kind, n_mols, h, depth, sdtype = WORKLOADS[args.workload]
    bf16 = sdtype == "bf16"
    torch.manual_seed(0)
    batch = make_batch(kind, n_mols, seed=1000 + env.rank)
    G = batch.collate("nodes")
    embedding = GraphEmbedding(42, 13, h)  # same RNG draws as two EmbeddingBag(42|13, h) in order
    with torch.no_grad():
        Xv, Xe = embedding.node(G.node_feats), embedding.edge(G.edge_feats)
    block = ChempropBlock(hidden_dim=h, depth=depth).eval()
    readout = Sum()
    if bf16:  # bf16 storage: the CPU baseline runs the fp32 oracle on the same bf16-rounded values
        block = block.to(torch.bfloat16)
        embedding = embedding.to(torch.bfloat16)
        Xv, Xe = Xv.to(torch.bfloat16), Xe.to(torch.bfloat16)
    Ws = [l.linear.weight.detach().float().clone() for l in block._chemprop_layers()]
    bs = [l.linear.bias.detach().float().clone() for l in block._chemprop_layers()]
    block = block.to(dev)
    Gd = G.update(node_feats=Xv, edge_feats=Xe).to(dev)
    Xv, Xe = Xv.float(), Xe.float()
    V, E, B = G.num_nodes, G.num_edges, len(G)
    torch.cuda.synchronize(dev)

    def step():
        out = block(Gd)
        return readout(out)

    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        events = []
        _engine.UPDATE_EVENTS = events
        if env.distributed:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        if env.distributed:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        _engine.UPDATE_EVENTS = None

    # Second, smaller measurement (not `value`): the whole encoder from the collated type indices,
    # GraphEmbedding fused into the initial gather (EmbeddedChempropBlock) + Sum readout.
    embedded = None
    if not args.no_embedded:
        Graw = batch.collate("nodes").to(dev)
        embedded = {
            "step": "GraphEmbedding + ChempropBlock + Sum from the collated integer type indices "
                    "(EmbeddedChempropBlock; fused = embedding folded into the initial gather, "
                    "unfused = nt_embed_bag kernels then the block)",
            "unit": "edge-messages/s",
        }
        for fuse in (True, False):
            enc = EmbeddedChempropBlock(embedding, block, fuse=fuse).eval().to(dev)
            with torch.no_grad():
                for _ in range(max(2, args.warmup // 2)):
                    readout(enc(Graw))
                if env.distributed:
                    dist.barrier()
                torch.cuda.synchronize(dev)
                t1 = time.perf_counter()
                for _ in range(args.steps):
                    readout(enc(Graw))
                torch.cuda.synchronize(dev)
                if env.distributed:
                    dist.barrier()
                e_el = time.perf_counter() - t1
            _, e_secs, e_rate = aggregate_throughput(E * depth * args.steps, e_el, device=dev)
            tag = "fused" if fuse else "unfused"
            embedded[f"{tag}_ms_per_step"] = e_secs / args.steps * 1e3
            embedded[f"{tag}_value"] = e_rate

    # Third (reported separately, never `value`): end to end from host Graph objects —
    # native collate on the host, H2D copy (pageable), then the fused embedded encoder + readout.
    end_to_end = None
    if not args.no_embedded and env.rank == 0:
        from notorch_amd.data.models.graph import BatchedGraph

        graphs = batch.to_graphs()
        enc = EmbeddedChempropBlock(embedding, block, fuse=True).eval().to(dev)
        parts = {"collate": [], "h2d": [], "device": []}
        with torch.no_grad():
            for it in range(6):
                torch.cuda.synchronize(dev)
                t_a = time.perf_counter()
                Gh = BatchedGraph.from_graphs(graphs)
                t_b = time.perf_counter()
                Gdev = Gh.to(dev)
                torch.cuda.synchronize(dev)
                t_c = time.perf_counter()
                readout(enc(Gdev))
                torch.cuda.synchronize(dev)
                t_d = time.perf_counter()
                if it:  # the first pass builds caches
                    parts["collate"].append(t_b - t_a)
                    parts["h2d"].append(t_c - t_b)
                    parts["device"].append(t_d - t_c)
        med = {k: statistics.median(v) * 1e3 for k, v in parts.items()}
        total = sum(med.values())
        end_to_end = {
            "step": f"{B} host Graphs -> BatchedGraph.from_graphs (native collate) -> .to(device) "
                    "(pageable H2D) -> EmbeddedChempropBlock + Sum; rank 0, median of 5",
            "collate_ms": med["collate"], "h2d_ms": med["h2d"], "device_ms": med["device"],
            "total_ms": total, "value": E * depth / (total * 1e-3), "unit": "edge-messages/s",
        }

    from notorch_amd import kernels as K

    lay = getattr(Gd, "_nt_layout", None)
    used_fused = bool(
        lay is not None and _engine._fused_enabled() and K.fused_supported(V, E, h, Gd.edge_feats.dtype)
        and _engine.fused_plan(lay, V, E) is not None
    )
    upd_ms = statistics.mean(a.elapsed_time(b) for a, b in events)
    units, secs, rate = aggregate_throughput(E * depth * args.steps, elapsed, device=dev)
    if env.rank != 0:
        if env.distributed:
            dist.destroy_process_group()
        return

    flops_upd = 2 * E * h * h
    upd_bytes = update_bytes(V, E, h)
    variant = os.environ.get("NT_UPDATE_KERNEL", "as")
    fused = used_fused
    persistent = (not fused and not bf16 and _engine._fused_enabled()
                  and K.fused_supported(V, E, h, Gd.edge_feats.dtype))
    traffic = read_pmc_traffic(args.pmc_csv) if args.pmc_csv else None
    if bf16:
        # native bf16 MFMA (16x16x32, K padded to 32, N to 16); HBM bytes at 2 B per element
        kp, np_ = 32 * ((h + 31) // 32), 16 * ((h + 15) // 16)
        upd_bytes = update_bytes(V, E, h, b=2)
        bf16_flops = 2 * E * kp * np_
        t_hbm = upd_bytes / (PEAK_HBM_GBPS * 1e9)
        t_mfma = bf16_flops / (PEAK_BF16_MFMA_TFLOPS * 1e12)
        bound = "hbm" if t_hbm >= t_mfma else "mfma"
        if bound == "hbm":
            achieved, peak, unit = upd_bytes / (upd_ms * 1e-3) / 1e9, PEAK_HBM_GBPS, "GB/s"
        else:
            achieved, peak, unit = bf16_flops / (upd_ms * 1e-3) / 1e12, PEAK_BF16_MFMA_TFLOPS, "TFLOP/s"
        kname = "nt_dmpnn_update (update_bf16_kernel: 64-edge tiles, bf16 16x16x32 MFMA, fp32 accumulate)"
        extra = {
            "mfma_bf16_tflops": bf16_flops / (upd_ms * 1e-3) / 1e12,
            "mfma_bf16_frac": bf16_flops / (upd_ms * 1e-3) / 1e12 / PEAK_BF16_MFMA_TFLOPS,
            "hbm_frac": upd_bytes / (upd_ms * 1e-3) / 1e9 / PEAK_HBM_GBPS,
            "t_min_us": max(t_hbm, t_mfma) * 1e6,
        }
        x6 = False
    elif fused or persistent or (h % 4 == 0 and 97 <= h <= 512 and variant[0] in "axp"):
        # bf16x6 fp32 emulation: 6 bf16 MFMA products per fp32 product.  Fused / as16 kernels run
        # v_mfma_f32_16x16x32_bf16 (K padded to 32, N to 16); x6 runs 32x32x16 (K to 16, N to 32).
        if fused or persistent or variant[0] == "a":
            kp, np_ = 32 * ((h + 31) // 32), 16 * ((h + 15) // 16)
        else:
            kp, np_ = 16 * ((h + 15) // 16), 32 * ((h + 31) // 32)
        if fused:
            upd_bytes = fused_bytes(V, E, h)
            fk = os.environ.get("NT_FUSED_KERNEL", "pk")
            kname = ("nt_dmpnn_update_fused (update_%s_kernel: persistent producer/consumer, "
                     "bf16x6 16x16x32 MFMA, aggregation of the next layer fused)" % ("ps" if fk == "ps" else "pk"))
        elif persistent:
            kname = ("nt_dmpnn_update_fused without tile plan (update_pk_kernel, bf16x6 16x16x32 MFMA; "
                     "hub graph: aggregation by the chunked segment reduce)")
        else:
            kname = f"nt_dmpnn_update (bf16x6 variant {variant})"
        bf16_flops = 6 * 2 * E * kp * np_
        t_hbm = upd_bytes / (PEAK_HBM_GBPS * 1e9)
        t_mfma = bf16_flops / (PEAK_BF16_MFMA_TFLOPS * 1e12)
        bound = "hbm" if t_hbm >= t_mfma else "mfma"
        if bound == "hbm":
            achieved, peak, unit = upd_bytes / (upd_ms * 1e-3) / 1e9, PEAK_HBM_GBPS, "GB/s"
        else:
            achieved, peak, unit = bf16_flops / (upd_ms * 1e-3) / 1e12, PEAK_BF16_MFMA_TFLOPS, "TFLOP/s"
        extra = {
            "mfma_bf16_tflops": bf16_flops / (upd_ms * 1e-3) / 1e12,
            "mfma_bf16_frac": bf16_flops / (upd_ms * 1e-3) / 1e12 / PEAK_BF16_MFMA_TFLOPS,
            "hbm_frac": upd_bytes / (upd_ms * 1e-3) / 1e9 / PEAK_HBM_GBPS,
            "fp32_equiv_tflops": flops_upd / (upd_ms * 1e-3) / 1e12,
            "t_min_us": max(t_hbm, t_mfma) * 1e6,
        }
        x6 = True
    else:
        x6 = False
        bound = "mfma"
        achieved, peak, unit = flops_upd / (upd_ms * 1e-3) / 1e12, PEAK_FP32_MFMA_TFLOPS, "TFLOP/s"
        kname = "nt_dmpnn_update (fp32 16x16x4 MFMA, variant %s)" % variant
        extra = {"alg_hbm_gbps": upd_bytes / (upd_ms * 1e-3) / 1e9}
    fwd_bytes, fwd_flops = forward_bytes_flops(V, E, B, h, depth, b=2 if bf16 else 4)
    t_step = secs / args.steps
    mfma_peak = PEAK_BF16_MFMA_TFLOPS if bf16 else PEAK_FP32_MFMA_TFLOPS
    t_min = max(fwd_bytes / (PEAK_HBM_GBPS * 1e9), fwd_flops / (mfma_peak * 1e12))
    line = {
        "metric": METRIC,
        "value": rate,
        "unit": "edge-messages/s",
        "n_gpus": env.world_size,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t_step * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if bf16 else "f32",
        "mfma_numerics": ("bf16 MFMA, fp32 accumulate" if bf16 else
                          "bf16x6 split (fp32-accurate)" if x6 else "fp32 MFMA"),
        "data": f"synthetic (seeded {kind}-shaped molecules per rank, random-init EmbeddingBag + weights)",
        "config": {
            "workload": f"{args.workload}: {n_mols} {kind}-shaped molecules per GPU, D-MPNN depth={depth} "
            f"hidden={h}, ChempropBlock + Sum readout, reference collate (rev offset by nodes)",
            "molecules_per_gpu": n_mols,
            "V_per_gpu": V,
            "E_per_gpu": E,
            "hidden": h,
            "depth": depth,
            "parallelism": f"molecule-sharded x{env.world_size}, no collective on the forward path",
        },
        "roofline": {
            "kernel": kname,
            "bound": bound,
            "achieved": achieved,
            "peak": peak,
            "unit": unit,
            "frac": achieved / peak,
            "traffic": traffic,
            "launch_ms": upd_ms,
            "launches_timed": len(events),
            "alg_bytes_per_launch": upd_bytes,
            "flops_per_launch_fp32": flops_upd,
            "alg_hbm_gbps": upd_bytes / (upd_ms * 1e-3) / 1e9,
            **extra,
        },
        "embedded_encoder": embedded,
        "end_to_end": end_to_end,
        "forward_roofline": {
            "alg_bytes": fwd_bytes,
            "flops": fwd_flops,
            "hbm_frac": fwd_bytes / t_step / (PEAK_HBM_GBPS * 1e9),
            "mfma_frac": fwd_flops / t_step / (mfma_peak * 1e12),
            "binding_frac": t_min / t_step,
        },
    }
    if not args.no_cpu_baseline and env.world_size == 1:
        line["cpu_baseline"] = cpu_baseline(G, Xv, Xe, Ws, bs, depth, args.cpu_seconds)
    else:
        line["cpu_baseline"] = None
    print(json.dumps(line), flush=True)
    if env.distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
