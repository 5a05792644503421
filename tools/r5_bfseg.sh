#!/bin/bash
# bf16 segment reduce with 4 rows in flight ('') vs one row in flight per thread (variant ab0):
# bf16 tests, then the zinc-4096-bf16 secondary of bench.py
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_bf16_backward.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_bfseg_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_bfseg_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/r5_bfseg_tests.log | head; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for L in "" variant:ab0; do
  NT_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-embedded --no-training > gpurun_out/r5_bfseg.log 2>&1 || { tail -5 gpurun_out/r5_bfseg.log; exit 5; }
  echo "lib '$L': $(tail -1 gpurun_out/r5_bfseg.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["secondary"]["zinc-4096-bf16"]; print("zinc", round(s["ms_per_step"]*1e3,1), "us/step", round(s["roofline"]["launch_us"],1), "us/launch")')"
done; done
