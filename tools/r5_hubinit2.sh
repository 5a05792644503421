#!/bin/bash
# hub graphs: wave init for nodes of in-degree <= 32 + chunked init of the hubs alone; tests then
# polymer-16 bench lines
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_hubs.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_backward.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_hi2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_hi2_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/r5_hi2_tests.log | head; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --workload polymer-16 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r5_hi2.log 2>&1 || { tail -5 gpurun_out/r5_hi2.log; exit 5; }
  echo "polymer: $(tail -1 gpurun_out/r5_hi2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step", d["value"])')"
done
bash tools/r5_poly_trace.sh | head -12
