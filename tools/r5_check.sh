#!/bin/bash
# Round-5 checkpoint: the GPU test suite, smoke, the default bench line.
set -uo pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/r5_tests.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_smoke.log 2>&1 || { tail -5 gpurun_out/r5_smoke.log; exit 5; }
tail -1 gpurun_out/r5_smoke.log
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 600 python bench.py > gpurun_out/r5_bench.log 2>&1 || { tail -5 gpurun_out/r5_bench.log; exit 6; }
  tail -1 gpurun_out/r5_bench.log | cut -c1-600
fi
