"""bench.py — edge-messages/s of the D-MPNN forward (ChempropBlock + Sum readout) on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 launched by
``torch.distributed.run`` (one rank per GPU, RCCL only for bench bookkeeping).  Rank 0 prints ONE
JSON line.

Headline workload (BASELINE.json configs[1] = SURVEY §8(d) config 2): per GPU a 4096-molecule
QM9-shaped batch (synthetic, seeded per rank -> weak scaling), hidden 300, depth 3, fp32, ReLU,
residual, sum reduce, reference collate semantics (rev offset by nodes).  A "step" = one forward
of ChempropBlock + Sum readout with the collated graph (incl. its CSR layout) and the embedded
features already resident in HBM.  value = sum over ranks of E_r * depth * K / max over ranks of
the timed seconds.

Other workloads (``--workload``): ``qm9-1m-sharded`` is BASELINE config 4: ONE seeded
1,000,000-molecule batch cut into 8 edge-balanced contiguous shards (shard.edge_balanced_ranges);
rank r of N runs shards r, r + N, ... each as its own collated batch (N = 8: one 125k shard per
GPU; N = 1: all eight in turn) -> fixed total work ("strong").  ``zinc-4096-bf16`` is config 3,
``polymer-16`` config 5; both are also measured in every default run as ``secondary`` keys.

Also in the line:
* ``roofline`` for the dominant kernel (the fused layer update; per-launch duration from HIP events
  recorded on the launch stream around every launch inside the timed region), with SURVEY §8(d)'s
  definitions: ``frac`` = t_min / launch time, t_min = max(algorithmic bytes / 8 TB/s, the MFMA
  products the kernel issues / the peak of that MFMA type) -- the roof of the instructions it really
  runs (fp32 storage: 3 fp16 products per MAC at 2.5 PF, so HBM binds at h = 300); ``hbm_frac`` =
  algorithmic bytes / launch time / 8 TB/s; ``fp32_equiv_frac`` = 2·E·h² fp32 flops / launch time /
  157.3 TF, a throughput figure beside it; ``traffic`` = HBM bytes per launch from rocprofv3 FETCH_SIZE (x2,
  gfx950) + WRITE_SIZE, read from ``--pmc-csv`` or from the committed profile of this workload
  (labelled with the commit it was taken at);
* ``cpu_baseline``: the oracle restatement (ATen CPU) on the host, rank 0, N=1, a bounded sample,
  at P = 1 and at P = the box's CPU share;
* ``fresh_batch``: the same forward on never-seen collated graphs (CSR + plans shipped by the
  collate, no device->host sync), ``end_to_end``: host Graphs -> collate -> H2D -> forward.
"""
from __future__ import annotations

import argparse
import copy
import glob
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from notorch_amd.shard import aggregate_throughput, dist_env, edge_balanced_ranges  # noqa: E402

METRIC = "edge-messages/sec D-MPNN depth=3 h=300, QM9-shaped batches, 1/2/4/8 MI355X"
PEAK_FP32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense fp32 MFMA (= vector) peak
PEAK_HBM_GBPS = 8000.0
PEAK_16BIT_MFMA_TFLOPS = 2500.0  # dense bf16 / fp16 MFMA (MI355X_MICROARCH.md)

WORKLOADS = {
    # name: (generator, molecules, hidden, depth, storage dtype)
    "qm9-4096": ("qm9", 4096, 300, 3, "f32"),  # BASELINE config 2 (the metric's configuration)
    "qm9-8192": ("qm9", 8192, 300, 3, "f32"),  # batch-size sweep points (the fp32 layer's walk crossover)
    "qm9-16k": ("qm9", 16384, 300, 3, "f32"),
    "qm9-32k": ("qm9", 32768, 300, 3, "f32"),  # HBM-scale batch (working set >> Infinity Cache)
    "qm9-125k": ("qm9", 125000, 300, 3, "f32"),  # one GPU's 1M/8 shard size in one batch
    "qm9-1m-sharded": ("qm9v", 1_000_000, 300, 3, "f32"),  # BASELINE config 4 (see header)
    "zinc-4096-bf16": ("zinc", 4096, 512, 5, "bf16"),  # BASELINE config 3 (bf16)
    "zinc-4096": ("zinc", 4096, 512, 5, "f32"),  # config 3 shape, fp32
    "polymer-16": ("polymer", 16, 300, 3, "f32"),  # BASELINE config 5
}
SECONDARY = ("zinc-4096-bf16", "polymer-16")
N_SHARDS = 8  # config 4: 1M molecules over 8 MI355X


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--prewarm-s", type=float, default=1.0,
                   help="untimed steps for at least this long before the W warm-up steps: the GPU "
                        "reaches its sustained clock only after ~1 s of load (measured: the layer "
                        "kernel runs 115 us right after a cold start, 106-109 us at steady state)")
    p.add_argument("--workload", default="qm9-4096", choices=sorted(WORKLOADS))
    p.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU baseline budget per thread count")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--event-every", type=int, default=8,
                   help="the roofline's per-launch HIP events on every N-th step of the timed region (each "
                        "event record costs the step about 7 us, so recording every step would slow the "
                        "headline it sits in by about 5 %%)")
    p.add_argument("--no-embedded", action="store_true", help="skip embedded / fresh / end-to-end legs")
    p.add_argument("--no-secondary", action="store_true", help="skip the config-3 / config-5 keys")
    p.add_argument("--no-training", action="store_true", help="skip the training key (N=1 only)")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="process group for the bench bookkeeping (nccl = RCCL; gloo only to rehearse "
                   "the N>1 path with --same-device on a one-GPU box)")
    p.add_argument("--same-device", action="store_true",
                   help="every rank on cuda:0 (rehearsal of the N>1 code path on one GPU; not a "
                   "scaling measurement)")
    p.add_argument("--launch-check", action="store_true",
                   help="CPU check of the N-rank launch: ranks join a gloo group, all-reduce the "
                   "bookkeeping scalars and rank 0 prints n_gpus; no GPU work")
    p.add_argument("--pmc-csv", default=None,
                   help="comma-separated rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE counter CSVs of the "
                   "same command (tools/profile.sh) to fill roofline.traffic")
    return p.parse_args()


# --------------------------------------------------------------------------- roofline models
def forward_bytes_flops(V, E, B, h, d, b=4):
    """SURVEY §8(d) minimal-traffic model of the fused forward + its MFMA flops."""
    rows = b * h * ((2 * d + 3) * (E + V) + B)
    idx = 4 * ((3 * d + 2) * E + (d + 1) * (V + 1) + (B + 1))
    wts = d * (h * h + h) * b
    return rows + idx + wts, 2 * d * E * h * h


def fused_bytes(V, E, h, b=4):
    """Algorithmic bytes of ONE fused layer launch (SURVEY §8(d) minimal model of a layer: read H,
    read S, write H', write S' = 2E + 2V rows; int32 src/rev/perm; weights once)."""
    return b * h * (2 * E + 2 * V) + 4 * 3 * E + (h * h + h) * b


def update_bytes(V, E, h, b=4):
    """Algorithmic bytes of ONE unfused update launch: read H[e], gather S[src[e]] and H[rev[e]],
    write H_out[e] (4 rows per edge), src + rev int64, weights once."""
    return 4 * E * h * b + 16 * E + (h * h + h) * b


# --------------------------------------------------------------------------- workloads
class Job:
    """One collated batch resident on the device, ready for block(Gd)."""

    def __init__(self, batch, G, Gd, h, depth, bf16):
        self.batch, self.G, self.Gd = batch, G, Gd
        self.V, self.E, self.B = G.num_nodes, G.num_edges, len(G)
        self.h, self.depth, self.bf16 = h, depth, bf16


def make_model(h, depth, bf16, dev):
    from notorch_amd.nn import ChempropBlock, GraphEmbedding

    torch.manual_seed(0)
    embedding = GraphEmbedding(42, 13, h)  # same RNG draws as two EmbeddingBag(42|13, h) in order
    block = ChempropBlock(hidden_dim=h, depth=depth).eval()
    if bf16:
        block = block.to(torch.bfloat16)
        embedding = embedding.to(torch.bfloat16)
    return embedding.to(dev), block.to(dev)


def embed_on_device(embedding, G, dev):
    """Collated type indices -> device, embedded by the GraphEmbedding kernel (nt_embed_bag)."""
    Gt = copy.copy(G).to(dev)  # Graph.to moves in place: keep the host graph for the CPU baseline
    with torch.no_grad():
        return embedding(Gt)


def make_jobs(name, rank, world, dev, embedding):
    from notorch_amd.data.synth import make_batch, make_qm9_batch_vectorized

    kind, n_mols, h, depth, sdtype = WORKLOADS[name]
    bf16 = sdtype == "bf16"
    jobs = []
    if kind == "qm9v":
        full = make_qm9_batch_vectorized(n_mols, seed=1000)
        ranges = edge_balanced_ranges(2 * full.n_bonds, N_SHARDS)
        for i in range(rank, N_SHARDS, world):
            sub = full.subset(*ranges[i])
            G = sub.collate("nodes")
            jobs.append(Job(sub, G, embed_on_device(embedding, G, dev), h, depth, bf16))
        return jobs, full, ranges
    batch = make_batch(kind, n_mols, seed=1000 + rank)
    G = batch.collate("nodes")
    jobs.append(Job(batch, G, embed_on_device(embedding, G, dev), h, depth, bf16))
    return jobs, batch, None


def prewarm(step, seconds, dev):
    """Untimed steps until `seconds` of wall time have passed (synchronised in rounds of 8 steps):
    the clock-settling phase before the counted warm-up steps; returns the steps it ran."""
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(8):
            step()
        n += 8
        torch.cuda.synchronize(dev)
    return n


def timed_steps(step, steps, warmup, env, dev):
    with torch.no_grad():
        for _ in range(warmup):
            step()
        if env.distributed:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize(dev)
        if env.distributed:
            dist.barrier()
        return time.perf_counter() - t0


def issue_model(engine_info, bf16):
    """(MFMA products per fp32 MAC, the peak those products issue at): the instructions the layer
    kernel actually issues, so that the roof is the one it sits under.  fp32 storage runs the scaled
    two-part fp16 split (3 fp16 products per MAC, 16-bit MFMA peak) unless the engine reports the
    exact fp32 MFMA path; bf16 storage issues one bf16 product per MAC."""
    products = engine_info.get("products", 1)
    exact_f32 = not bf16 and products == 1
    return products, PEAK_FP32_MFMA_TFLOPS if exact_f32 else PEAK_16BIT_MFMA_TFLOPS


def launch_roofline(jobs, events, engine_info, traffic, traffic_src):
    """Roofline of the dominant kernel (the layer update) from the per-launch HIP events.

    The binding roof is the larger of t_hbm = algorithmic bytes / 8 TB/s and t_mfma = the MFMA
    products the kernel issues / the peak of that MFMA type; ``frac`` = t_min / launch
    time, so it can never exceed 1.  The fp32-equivalent throughput (2·E·h² fp32 flops per launch over
    the fp32 MFMA peak) is reported beside it as ``fp32_equiv_frac``: a throughput figure, not a roof
    (the kernel issues no fp32 MFMA)."""
    upd_ms = statistics.mean(a.elapsed_time(b) for a, b in events)
    t = upd_ms * 1e-3
    j = max(jobs, key=lambda x: x.E)
    V, E, h = j.V, j.E, j.h
    b = 2 if j.bf16 else 4
    fused = engine_info.get("fused", False)
    alg_bytes = fused_bytes(V, E, h, b) if fused else update_bytes(V, E, h, b)
    flops = 2 * E * h * h
    kp, np_ = engine_info.get("kpad", h), engine_info.get("npad", h)
    products, mfma_peak = issue_model(engine_info, j.bf16)
    issued = products * 2 * E * kp * np_
    t_hbm = alg_bytes / (PEAK_HBM_GBPS * 1e9)
    t_mfma = issued / (mfma_peak * 1e12)
    t_min = max(t_hbm, t_mfma)
    hbm_gbps = alg_bytes / t / 1e9
    out = {"kernel": engine_info.get("kernel", "?"), "numerics": engine_info.get("numerics", "?")}
    if t_hbm >= t_mfma:
        out.update(bound="hbm", achieved=hbm_gbps, peak=PEAK_HBM_GBPS, unit="GB/s")
    else:
        out.update(bound="mfma", achieved=issued / t / 1e12, peak=mfma_peak, unit="TFLOP/s")
    out.update(
        frac=t_min / t,
        traffic=traffic, traffic_source=traffic_src,
        traffic_over_alg=None if traffic is None else traffic / alg_bytes,
        launch_us=upd_ms * 1e3, launches_timed=len(events),
        alg_bytes_per_launch=alg_bytes, flops_per_launch_fp32=flops,
        hbm_frac=hbm_gbps / PEAK_HBM_GBPS, alg_hbm_gbps=hbm_gbps,
        mfma_issued_per_launch=issued, mfma_issue_peak_tflops=mfma_peak,
        mfma_issue_tflops=issued / t / 1e12, mfma_issue_frac=issued / t / 1e12 / mfma_peak,
        t_hbm_us=t_hbm * 1e6, t_mfma_us=t_mfma * 1e6, t_min_us=t_min * 1e6,
    )
    if not j.bf16:
        out.update(fp32_equiv_tflops=flops / t / 1e12, fp32_equiv_frac=flops / t / 1e12 / PEAK_FP32_MFMA_TFLOPS)
    return out


# --------------------------------------------------------------------------- PMC traffic
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


def committed_traffic(workload, kernel_substr):
    """Traffic per launch from the newest committed profile of this workload (profiles/*/<workload>/
    PMC.json, written by tools/save_profile.py from the same command's --pmc passes)."""
    best = None
    for f in glob.glob(os.path.join(ROOT, "profiles", "*", workload, "PMC.json")):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if kernel_substr in d.get("kernel", "") and (best is None or d.get("time", 0) > best[0].get("time", 0)):
            best = (d, f)
    if best is None:
        return None, None
    d, f = best
    return d["traffic_per_launch"], f"rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, builder-profiled at {d['commit']} " \
        f"({os.path.relpath(f, ROOT)})"


# --------------------------------------------------------------------------- CPU baseline
def cpu_baseline(job, embedding, budget_s, sample_mols=4096):
    """Oracle restatement (ATen CPU) timed on the host at P = 1, at P = the box's CPU share
    (OMP_NUM_THREADS, which the GPU box sets to its per-GPU share) and at P = the physical cores this
    process may run on (lscpu cores, capped at the affinity mask), median of runs per budget; the
    reported value is the fastest P."""
    from oracle import dmpnn_ref

    if job.B > sample_mols:  # bounded sample: the first sample_mols molecules of the job
        G = job.batch.subset(0, sample_mols).collate("nodes")
        sample = f"first {sample_mols} molecules of the job's batch"
    else:
        G = job.G
        sample = f"the same {job.B}-molecule batch"
    emb = copy.deepcopy(embedding).float().cpu()
    blk_Ws, blk_bs = WS_BS
    with torch.no_grad():
        Xv, Xe = emb.node(G.node_feats), emb.edge(G.edge_feats)
        if job.bf16:  # the fp32 oracle on the bf16-rounded values the device path stores
            Xv, Xe = Xv.to(torch.bfloat16).float(), Xe.to(torch.bfloat16).float()
    ei, rev, bni, B = G.edge_index, G.rev_index, G.batch_node_index, len(G)
    try:
        visible = len(os.sched_getaffinity(0))
    except AttributeError:
        visible = os.cpu_count() or 1
    share = min(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or 16, visible)
    host = host_cpu_info()
    # P = 1, the box's per-GPU CPU share, and P = the physical cores this process may use (the
    # BASELINE.md plan: set_num_threads(P) with P = the physical cores); value = the fastest P
    phys = min(host.get("physical_cores", visible) or visible, visible)
    thread_counts = sorted({1, share, phys})

    def one():
        with torch.inference_mode():
            n, _ = dmpnn_ref.chemprop_block(Xv, Xe, ei, rev, blk_Ws, blk_bs)
            dmpnn_ref.readout(n, bni, B, "sum")

    res = {}
    prev = torch.get_num_threads()
    for P in thread_counts:
        torch.set_num_threads(P)
        one()  # warm-up
        times, t_start = [], time.perf_counter()
        while (time.perf_counter() - t_start < budget_s and len(times) < 200) or len(times) < 3:
            t0 = time.perf_counter()
            one()
            times.append(time.perf_counter() - t0)
        res[P] = (statistics.median(times), len(times))
    torch.set_num_threads(prev)
    E = ei.shape[1]
    best_P = min(res, key=lambda p: res[p][0])
    return {
        "value": E * job.depth / res[best_P][0],
        "unit": "edge-messages/s",
        "cores": best_P,
        "kind": "port",
        "by_threads": {str(p): {"value": E * job.depth / m, "ms": m * 1e3, "runs": n} for p, (m, n) in res.items()},
        "host": dict(host, cpus_visible=visible),
        "sample": f"oracle/dmpnn_ref.py (ATen CPU restatement of chemprop.py+agg.py) on {sample} "
        f"(V={G.num_nodes}, E={E}), fp32, torch.set_num_threads(P) for P in {sorted(res)} (P = 1, "
        f"the box's per-GPU CPU share OMP_NUM_THREADS={share} and the physical cores usable here, {phys}); "
        f"host {host.get('model', '?')}, "
        f"{host.get('physical_cores', '?')} physical cores ({visible} CPUs visible to this process); "
        f"median of runs within {budget_s:.0f} s each after 1 warm-up; value and cores = the fastest P",
    }


def host_cpu_info():
    """Physical core count and model of the host (lscpu), for the cpu_baseline's `cores` context."""
    import subprocess

    info = {}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
    except (OSError, subprocess.SubprocessError):
        return info
    kv = {}
    for line in out.splitlines():
        if ":" in line:
            k, v = line.split(":", 1)
            kv[k.strip()] = v.strip()
    try:
        info["physical_cores"] = int(kv["Core(s) per socket"]) * int(kv["Socket(s)"])
        info["threads_per_core"] = int(kv.get("Thread(s) per core", "1"))
    except (KeyError, ValueError):
        pass
    if "Model name" in kv:
        info["model"] = kv["Model name"]
    return info


WS_BS = None  # (weights, biases) of the headline block on the host, for the CPU baseline
BOOK_DEV = None  # device of the bookkeeping all-reduce tensors (the GPU under RCCL, cpu under gloo)


# --------------------------------------------------------------------------- main
def run_workload(name, args, env, dev, headline):
    from notorch_amd.nn import Sum
    from notorch_amd.nn.gnn import _engine

    kind, n_mols, h, depth, sdtype = WORKLOADS[name]
    bf16 = sdtype == "bf16"
    embedding, block = make_model(h, depth, bf16, dev)
    jobs, batch, ranges = make_jobs(name, env.rank, env.world_size, dev, embedding)
    readout = Sum()
    torch.cuda.synchronize(dev)

    events = []
    # at least two sampled steps, at most one in `event_every`, none at the region's edges
    every = max(1, args.event_every, args.steps // 2)
    offset = max(0, min(every // 2, args.steps - 1))
    count = [0]

    def step():
        # the per-launch roofline events ride on the steps i = offset mod every of the timed region;
        # the others run exactly as a user's forward does
        _engine.UPDATE_EVENTS = events if count[0] % every == offset else None
        count[0] += 1
        for j in jobs:
            readout(block(j.Gd))

    with torch.no_grad():
        prewarm(step, args.prewarm_s, dev)
        for _ in range(args.warmup):
            step()
    events.clear()
    count[0] = 0
    elapsed = timed_steps(step, args.steps, 0, env, dev)
    _engine.UPDATE_EVENTS = None
    info = dict(_engine.LAST_UPDATE_INFO)
    E_rank = sum(j.E for j in jobs)
    units, secs, rate = aggregate_throughput(E_rank * depth * args.steps, elapsed, device=BOOK_DEV)
    res = {"jobs": jobs, "embedding": embedding, "block": block, "readout": readout, "events": events,
           "event_every": every, "event_offset": offset,
           "info": info, "units": units, "secs": secs, "rate": rate, "batch": batch, "ranges": ranges,
           "name": name, "kind": kind, "h": h, "depth": depth, "bf16": bf16, "n_mols": n_mols,
           "steps": args.steps}
    if headline:
        global WS_BS
        layers = block._chemprop_layers()
        WS_BS = ([l.linear.weight.detach().float().cpu().clone() for l in layers],
                 [l.linear.bias.detach().float().cpu().clone() for l in layers])
    return res


def fresh_batch_leg(res, args, env, dev, n_fresh=6):
    """Forward on graphs the engine has never seen (collated on the host, CSR + plans shipped)."""
    job = res["jobs"][0]
    block, readout = res["block"], res["readout"]
    Xv, Xe = job.Gd.node_feats, job.Gd.edge_feats
    fresh = [job.batch.collate("nodes").to(dev).update(node_feats=Xv, edge_feats=Xe) for _ in range(n_fresh + 1)]
    torch.cuda.synchronize(dev)
    with torch.no_grad():
        readout(block(fresh[0]))  # first call of the process for this shape (allocator, packs)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for G in fresh[1:]:
            readout(block(G))
        torch.cuda.synchronize(dev)
        t = (time.perf_counter() - t0) / n_fresh
    resident = res["secs"] / args.steps / len(res["jobs"])
    return {"step": f"{n_fresh} never-seen collated graphs (host CSR + tile plan shipped by the collate), "
                    "resident features, back to back", "fresh_batch_ms": t * 1e3,
            "resident_ms": resident * 1e3, "ratio": t / resident}


def embedded_leg(res, args, env, dev):
    from notorch_amd.nn import EmbeddedChempropBlock

    job = res["jobs"][0]
    Graw = copy.copy(job.G).to(dev)
    out = {"step": "GraphEmbedding + ChempropBlock + Sum from the collated integer type indices "
                   "(EmbeddedChempropBlock; fused = embedding folded into the initial gather, "
                   "unfused = nt_embed_bag kernels then the block)", "unit": "edge-messages/s"}
    for fuse in (True, False):
        enc = EmbeddedChempropBlock(res["embedding"], res["block"], fuse=fuse).eval()
        el = timed_steps(lambda: res["readout"](enc(Graw)), args.steps, max(2, args.warmup // 2), env, dev)
        _, e_secs, e_rate = aggregate_throughput(job.E * job.depth * args.steps, el, device=BOOK_DEV)
        tag = "fused" if fuse else "unfused"
        out[f"{tag}_ms_per_step"] = e_secs / args.steps * 1e3
        out[f"{tag}_value"] = e_rate
    return out


def end_to_end_leg(res, dev):
    from notorch_amd.data.models.graph import BatchedGraph
    from notorch_amd.nn import EmbeddedChempropBlock

    job = res["jobs"][0]
    graphs = job.batch.to_graphs()
    enc = EmbeddedChempropBlock(res["embedding"], res["block"], fuse=True).eval()
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
            res["readout"](enc(Gdev))
            torch.cuda.synchronize(dev)
            t_d = time.perf_counter()
            if it:  # the first pass builds caches
                parts["collate"].append(t_b - t_a)
                parts["h2d"].append(t_c - t_b)
                parts["device"].append(t_d - t_c)
    med = {k: statistics.median(v) * 1e3 for k, v in parts.items()}
    total = sum(med.values())
    return {"step": f"{job.B} host Graphs -> BatchedGraph.from_graphs (native collate) -> .to(device) "
                    "(pageable H2D) -> EmbeddedChempropBlock + Sum; rank 0, median of 5, serial",
            "collate_ms": med["collate"], "h2d_ms": med["h2d"], "device_ms": med["device"],
            "total_ms": total, "value": job.E * job.depth / (total * 1e-3), "unit": "edge-messages/s"}


def pipeline_leg(res, dev, workers, prefetch=3):
    """Steady-state host feed: per-molecule Graphs -> DataLoader workers (native collate, CSR and
    tile plan) -> pinned batches -> H2D on a side stream overlapped with the previous batch's
    EmbeddedChempropBlock + Sum (notorch_amd.data.loader.graph_loader: GraphFeeder workers collating
    into a page-locked slot ring).  The workers fill workers x slots batches ahead; the timed batches
    start after that many (+ 4) have been consumed, so they are collated at the workers' steady rate,
    not drained from the initial burst."""
    from notorch_amd.data.loader import graph_loader
    from notorch_amd.nn import EmbeddedChempropBlock

    job = res["jobs"][0]
    graphs = job.batch.to_graphs()
    B = len(graphs)
    warm = workers * prefetch + 4
    n_batches = warm + 3 * workers
    dataset = graphs * n_batches  # the same molecules every batch (references, no copies)
    enc = EmbeddedChempropBlock(res["embedding"], res["block"], fuse=True).eval()
    loader = graph_loader(dataset, B, dev, num_workers=workers, ring_slots=prefetch)
    with torch.no_grad():
        it = iter(loader)
        for _ in range(warm):
            res["readout"](enc(next(it)))
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        n = 0
        for G in it:
            res["readout"](enc(G))
            n += 1
        torch.cuda.synchronize(dev)
        t = (time.perf_counter() - t0) / max(n, 1)
    if hasattr(loader.batches, "close"):
        loader.batches.close()
    del loader, it
    device_ms = res["secs"] / res["steps"] / len(res["jobs"]) * 1e3
    return {"step": f"{B} host Graphs per batch -> GraphFeeder({workers} forked workers, native collate "
                    f"into {prefetch} page-locked ring slots each) -> side-stream DMA overlapped with the "
                    "previous batch's EmbeddedChempropBlock + Sum; steady state over "
                    f"{n} batches after {warm} (workers x slots + 4: the initial burst consumed)",
            "workers": workers, "ms_per_batch": t * 1e3,
            "device_step_ms": device_ms, "ratio_to_device_step": t * 1e3 / device_ms,
            "value": job.E * job.depth / t, "unit": "edge-messages/s"}


def training_leg(args, timeout_s=300):
    """Training steps as the reference trains (tools/train_bench.py --json, each in a fresh child
    process: zero_grad + forward + backward + Adam(lr=1e-4).step(), 10 warm-ups and at least 1 s
    more; 50 steps back to back in rounds of 10 between two events, the median round per step).  Headline: config 2 on the default (kernel) weight-grad
    path; `library` is the same step with NT_WGRAD=library, a comparison only; `config3_bf16` is
    config 3 (zinc-4096, bf16, h=512, depth=5) on the default path."""
    import subprocess

    script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools", "train_bench.py")
    out = {"step": "config 2 batch (4096 qm9-shaped molecules, seed 1000), ChempropBlock depth=3 h=300 + Sum, "
                   "zero_grad + forward + backward of sum(readout^2) w.r.t. weights and input features + "
                   "Adam(lr=1e-4).step() (model.py:153,273), fp32; fresh process per leg; 50 steps back to back "
                   "(no host sync between steps, as a training loop runs) in rounds of 10, median round per "
                   "step, after 10 warm-ups and >= 1 s of warm-up steps",
           "unit": "edge-messages/s"}

    def run(env_extra, extra_args):
        env = dict(os.environ, **env_extra)
        try:
            r = subprocess.run([sys.executable, script, "--json", "--modes", "kernel", "--steps", "50",
                                "--warmup", "10", "--warmup-s", "1", *extra_args], env=env,
                               capture_output=True, text=True, timeout=timeout_s)
        except subprocess.TimeoutExpired:
            return {"error": f"timed out after {timeout_s} s"}
        if r.returncode != 0:
            return {"error": f"exit {r.returncode}: {r.stderr.strip().splitlines()[-1:]}"}
        d = json.loads(r.stdout.strip().splitlines()[-1])
        return {"train_ms": d["ms"]["train[kernel]"], "forward_ms": d["ms"]["fwd"],
                "value": d["edge_messages_per_s"]["train[kernel]"]}

    out["kernel"] = run({}, [])
    out["library"] = run({"NT_WGRAD": "library"}, [])
    # the same step with torch's fused Adam implementation (one optimizer kernel instead of torch's
    # default foreach kernels, about 0.1 ms of tiny launches at config 2): a comparison, not the headline
    out["kernel_adam_fused"] = run({}, ["--optim", "adam-fused"])
    if "train_ms" in out["kernel"]:
        out.update(weight_grad="kernel", train_ms=out["kernel"]["train_ms"], value=out["kernel"]["value"])
    out["config3_bf16"] = dict(run({}, ["--kind", "zinc", "--h", "512", "--depth", "5", "--dtype", "bf16"]),
                               step="config 3 batch (4096 zinc-shaped molecules), depth=5 h=512, bf16 storage, "
                                    "same step (Adam included)")
    return out


def summary(res, args, env, pmc_csv=None):
    jobs = res["jobs"]
    info = res["info"]
    kern = info.get("kernel_short", "update")
    if pmc_csv:
        traffic, tsrc = read_pmc_traffic(pmc_csv, kern), "rocprofv3 --pmc of this command (--pmc-csv)"
    else:
        traffic, tsrc = committed_traffic(res["name"], kern)
    roof = launch_roofline(jobs, res["events"], info, traffic, tsrc)
    roof["launch_sampling"] = (f"HIP events on the launch stream around every layer launch of the steps "
                               f"i = {res['event_offset']} mod {res['event_every']} of the timed region "
                               f"({len(res['events'])} launches)")
    t_step = res["secs"] / args.steps
    V = sum(j.V for j in jobs)
    E = sum(j.E for j in jobs)
    B = sum(j.B for j in jobs)
    fwd_bytes, fwd_flops = forward_bytes_flops(V, E, B, res["h"], res["depth"], b=2 if res["bf16"] else 4)
    # the same binding-roof model as the layer roofline: bytes at 8 TB/s against the MFMA products the
    # kernels issue (padded k / n, 3 fp16 products per fp32 MAC) at that MFMA type's peak
    products, mfma_peak = issue_model(info, res["bf16"])
    kp, np_ = info.get("kpad", res["h"]), info.get("npad", res["h"])
    fwd_issued = products * 2 * res["depth"] * E * kp * np_
    t_min = max(fwd_bytes / (PEAK_HBM_GBPS * 1e9), fwd_issued / (mfma_peak * 1e12))
    return roof, {
        "alg_bytes_per_rank": fwd_bytes, "flops_per_rank": fwd_flops, "mfma_issued_per_rank": fwd_issued,
        "hbm_frac": fwd_bytes / t_step / (PEAK_HBM_GBPS * 1e9),
        "mfma_issue_frac": fwd_issued / t_step / (mfma_peak * 1e12),
        "binding_frac": t_min / t_step,
        "t_min_us": t_min * 1e6,
    }


def launch_check(args, env):
    """--launch-check: the rank bookkeeping of an N-rank run without a GPU (gloo): every rank joins
    the group, the units / max-time all-reduces run, rank 0 prints the line's rank fields."""
    if env.distributed:
        dist.init_process_group("gloo")
    units, secs, rate = aggregate_throughput(1000.0 * (env.rank + 1), 1.0 + env.rank)
    if env.rank == 0:
        print(json.dumps({"n_gpus": env.world_size, "value": rate, "units": units, "max_seconds": secs,
                          "launch_check": True}), flush=True)
    if env.distributed:
        dist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N` without a launcher: start the N rank processes here, before
        # anything touches the GPU (children, never an exec), and exit with their status.
        from notorch_amd.shard import launch_local_ranks

        sys.exit(launch_local_ranks([os.path.abspath(__file__), *sys.argv[1:]], args.gpus))
    env = dist_env()
    if env.world_size != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env.world_size} ranks were launched")
    if args.launch_check:
        return launch_check(args, env)
    dev = torch.device("cuda", 0 if args.same_device else env.local_rank)
    if env.distributed:
        torch.cuda.set_device(dev)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    global BOOK_DEV
    BOOK_DEV = dev if args.dist_backend == "nccl" else torch.device("cpu")

    from notorch_amd import _lib

    _lib.load()  # fail loudly if the HIP extension is missing
    res = run_workload(args.workload, args, env, dev, headline=True)
    job = res["jobs"][0]
    fresh = embedded = e2e = None
    if not args.no_embedded and res["kind"] != "qm9v":
        fresh = fresh_batch_leg(res, args, env, dev)
        embedded = embedded_leg(res, args, env, dev)
        if env.rank == 0:
            e2e = end_to_end_leg(res, dev)
            try:
                share = len(os.sched_getaffinity(0))
            except AttributeError:
                share = os.cpu_count() or 4
            share = min(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or share, share, 16)
            e2e["pipelined"] = pipeline_leg(res, dev, workers=max(4, share - 2))
    roof, fwd = summary(res, args, env, args.pmc_csv)

    secondary = None
    if not args.no_secondary and args.workload == "qm9-4096":
        secondary = {}
        for name in SECONDARY:
            r2 = run_workload(name, args, env, dev, headline=False)
            roof2, fwd2 = summary(r2, args, env)
            secondary[name] = {
                "config": f"{r2['n_mols']} {r2['kind']}-shaped molecules per GPU, depth={r2['depth']} "
                          f"hidden={r2['h']}, {'bf16' if r2['bf16'] else 'f32'}",
                "value": r2["rate"], "unit": "edge-messages/s", "ms_per_step": r2["secs"] / args.steps * 1e3,
                "V_per_gpu": r2["jobs"][0].V, "E_per_gpu": r2["jobs"][0].E,
                "roofline": roof2, "forward_roofline": fwd2,
            }
            del r2

    training = None
    if not args.no_training and env.world_size == 1 and args.workload == "qm9-4096":
        training = training_leg(args)

    cpu = None
    if not args.no_cpu_baseline and env.rank == 0:
        cpu = cpu_baseline(job, res["embedding"], args.cpu_seconds)
    if env.rank == 0:
        sharded = res["kind"] == "qm9v"
        line = {
            "metric": METRIC,
            "value": res["rate"],
            "unit": "edge-messages/s",
            "n_gpus": env.world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "prewarm_s": args.prewarm_s,
            "ms_per_step": res["secs"] / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None,
            "dtype": "bf16" if res["bf16"] else "f32",
            "mfma_numerics": res["info"].get("numerics", "?"),
            "data": f"synthetic (seeded {res['kind']}-shaped molecules, random-init EmbeddingBag + weights)",
            "config": {
                "workload": (f"{args.workload}: {res['n_mols']} qm9-shaped molecules in {N_SHARDS} edge-balanced "
                             f"shards, rank r runs shards r, r+N, ...; D-MPNN depth={res['depth']} hidden={res['h']}"
                             if sharded else
                             f"{args.workload}: {res['n_mols']} {res['kind']}-shaped molecules per GPU, D-MPNN "
                             f"depth={res['depth']} hidden={res['h']}")
                + ", ChempropBlock + Sum readout, reference collate (rev offset by nodes)",
                "molecules_per_gpu": sum(j.B for j in res["jobs"]),
                "V_per_gpu": sum(j.V for j in res["jobs"]),
                "E_per_gpu": sum(j.E for j in res["jobs"]),
                "shards_on_rank0": len(res["jobs"]) if sharded else None,
                "hidden": res["h"],
                "depth": res["depth"],
                "parallelism": f"molecule-sharded x{env.world_size}, no collective on the forward path",
            },
            "roofline": roof,
            "forward_roofline": fwd,
            "secondary": secondary,
            "fresh_batch": fresh,
            "embedded_encoder": embedded,
            "end_to_end": e2e,
            "training": training,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if env.distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
