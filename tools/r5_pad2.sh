#!/bin/bash
# padded rows on hub graphs: hub / fused / parity tests, then polymer-16 and qm9-4096 bench lines
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_hubs.py tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_config4.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_pad2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_pad2_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/r5_pad2_tests.log | head; [ $rc -eq 0 ] || exit $rc
for P in 1 0 1 0; do
  NT_ROW_PAD=$P timeout -k 10 300 python bench.py --workload polymer-16 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r5_pad2.log 2>&1 || { tail -5 gpurun_out/r5_pad2.log; exit 5; }
  echo "polymer pad=$P: $(tail -1 gpurun_out/r5_pad2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step", round(d["roofline"]["launch_us"],1), "us/launch")')"
done
