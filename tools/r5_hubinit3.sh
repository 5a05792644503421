#!/bin/bash
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_hubs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_hi3_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_hi3_tests.log; grep -E "^FAILED|^ERROR|^E " gpurun_out/r5_hi3_tests.log | head; exit $rc
