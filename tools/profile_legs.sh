#!/bin/bash
# Kernel-level stats of the embedded-encoder / fresh-batch legs and of the training step (rocprofv3
# --kernel-trace --stats only; no counters).  Usage: tools/profile_legs.sh <tag>
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TAG=${1:-r2c}
OUT=gpurun_out/legs_${TAG}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/qm9-4096" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > "$OUT/qm9-4096.log" 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/qm9-32k" -o run -- python3 bench.py --workload qm9-32k --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > "$OUT/qm9-32k.log" 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/train" -o run -- python3 tools/train_bench.py > "$OUT/train.log" 2>&1 || exit 4
echo "legs $TAG done"
