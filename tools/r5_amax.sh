#!/bin/bash
# amax chain atomics: one pair per workgroup in the layer kernel and 1024-thread init blocks (default)
# against one pair per wave / 256-thread init blocks (variant ab0): parity tests, then bench lines
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fk.py tests/test_gpu_numerics.py tests/test_gpu_fused.py tests/test_gpu_hubs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_amax_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_amax_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/r5_amax_tests.log | head; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for L in "" variant:ab0; do
  NT_LIB=$L timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r5_amax.log 2>&1 || { tail -5 gpurun_out/r5_amax.log; exit 5; }
  echo "lib '$L': $(tail -1 gpurun_out/r5_amax.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,1), "us/step", round(d["roofline"]["launch_us"],1), "us/launch")')"
done; done
