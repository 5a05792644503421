#!/bin/bash
# the 128-row one-workgroup walk against the 64-row two-workgroup walk: time and memory-pipeline counters
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/prof_r6_walks
mkdir -p "$OUT"
for r in 1 2; do timeout -k 10 300 python tools/kbench.py --only fk_fused,fk_fused64 --rounds 7 2>&1 | grep -E "median" || exit 5; done
i=0
for K in fk_fused fk_fused64; do
while read -r G; do
  [ -z "$G" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G -T --output-format csv -d "$OUT/${K}_p$i" -o run -- python3 tools/kbench.py --only $K --rounds 3 > "$OUT/${K}_p$i.log" 2>&1 || echo "pass $i ($G) failed rc=$?"
done <<'GROUPS'
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_WRITE_TAGCONFLICT_STALL_CYCLES_sum
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
GRBM_GUI_ACTIVE GRBM_COUNT
GROUPS
done
python3 - <<'PY'
import csv, glob, collections
for K in ("fk_fused", "fk_fused64"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/prof_r6_walks/{K}_p*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "update_fk_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(K, {k: f"{sum(v)/len(v):.4g}" for k, v in sorted(agg.items())})
PY
