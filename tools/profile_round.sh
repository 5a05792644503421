#!/bin/bash
# Per-round profile package: for each workload, one rocprofv3 --kernel-trace --stats pass, separate
# --pmc passes (FETCH_SIZE, WRITE_SIZE, SQ_*), then a bench line whose roofline.traffic is read from
# those counter CSVs.  Usage: tools/profile_round.sh <tag> [workload ...]
set -uo pipefail
TAG=${1:-r1}; shift || true
WORKLOADS=${*:-qm9-4096 zinc-4096-bf16 qm9-32k}
for W in $WORKLOADS; do
  D=gpurun_out/prof_${TAG}_${W}
  tools/profile.sh "${TAG}_${W}" --workload "$W" || { echo "profile $W failed"; exit 3; }
  F=$(find "$D/fetch" -name "*counter_collection.csv" | head -1)
  Wr=$(find "$D/write" -name "*counter_collection.csv" | head -1)
  timeout -k 10 300 python bench.py --workload "$W" --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-embedded --no-training \
    --pmc-csv "$F,$Wr" > "$D/bench.log" 2>&1 || { tail -5 "$D/bench.log"; exit 4; }
  tail -1 "$D/bench.log" | cut -c1-400
done
