#!/bin/bash
# Profile bench.py with rocprofv3 on the GPU box: one kernel-trace/stats pass and separate PMC
# passes (counters never combined with trace domains).  Usage: tools/profile.sh <tag> [bench args]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TAG=${1:-r1}; shift || true
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-embedded --no-training $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$OUT/write" -o run -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -T --output-format csv -d "$OUT/sq" -o run -- python3 bench.py $ARGS > "$OUT/sq.log" 2>&1
echo "profile $TAG done"
