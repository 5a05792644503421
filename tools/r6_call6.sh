#!/bin/bash
# init over the row table: tests, kbench init vs init_rows, then bench lines
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_init_rows.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_hubs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_c6_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6_c6_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/r6_c6_tests.log | head; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do timeout -k 10 300 python tools/kbench.py --only init,init_rows --rounds 7 2>&1 | grep -E "median" || exit 5; done
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r6_c6.log 2>&1 || { tail -5 gpurun_out/r6_c6.log; exit 5; }
  echo "bench: $(tail -1 gpurun_out/r6_c6.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["ms_per_step"]*1e3,1), "us/step", round(r["launch_us"],1), "us/launch")')"
done


