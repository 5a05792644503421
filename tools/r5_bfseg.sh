#!/bin/bash
# bf16 segment reduce with 8 rows in flight: bf16 tests, zinc bench line
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_bf16_backward.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_bfseg_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_bfseg_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/r5_bfseg_tests.log | head; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bfseg -o run -- python3 bench.py --workload zinc-4096-bf16 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r5_bfseg.log 2>&1 || { tail -5 gpurun_out/r5_bfseg.log; exit 5; }
grep '^{"metric"' gpurun_out/r5_bfseg.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])'
head -6 gpurun_out/bfseg/run_kernel_stats.csv | cut -c1-120
