#!/bin/bash
# chunked reduce: 8 rows in flight in pass 1, 32 sub-ranges in pass 2 for few segments (default)
# against 4 / 8 (variant sc0): chunked tests, then polymer-16 bench lines
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_hubs.py tests/test_gpu_parity.py tests/test_gpu_readout.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_sc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_sc_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/r5_sc_tests.log | head; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for L in "" variant:sc0; do
  NT_LIB=$L timeout -k 10 300 python bench.py --workload polymer-16 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r5_sc.log 2>&1 || { tail -5 gpurun_out/r5_sc.log; exit 5; }
  echo "lib '$L': $(tail -1 gpurun_out/r5_sc.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step")')"
done; done
