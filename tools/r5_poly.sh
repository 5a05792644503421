#!/bin/bash
# chunked reduce / hub-graph checks, then the polymer-16 per-dispatch trace and bench line
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_hubs.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_readout.py tests/test_gpu_backward.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_poly_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_poly_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/r5_poly_tests.log | head; [ $rc -eq 0 ] || exit $rc
bash tools/r5_poly_trace.sh
