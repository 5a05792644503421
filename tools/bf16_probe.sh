#!/bin/bash
# bf16 (config 3) timing probe: fused vs unfused bench lines + a kernel-trace summary of the fused run.
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/bf16_probe
J='import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["launch_ms"], d["roofline"]["frac"])'
timeout -k 10 120 python bench.py --workload zinc-4096-bf16 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bf16_probe/fused.log 2>&1 || exit 3
python -c "$J" < gpurun_out/bf16_probe/fused.log
NT_FUSED=0 timeout -k 10 120 python bench.py --workload zinc-4096-bf16 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bf16_probe/unfused.log 2>&1 || exit 4
python -c "$J" < gpurun_out/bf16_probe/unfused.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/bf16_probe/trace -o run -- python3 bench.py --workload zinc-4096-bf16 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bf16_probe/trace.log 2>&1 || exit 5
f=$(find gpurun_out/bf16_probe/trace -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -12
