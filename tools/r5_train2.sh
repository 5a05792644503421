#!/bin/bash
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_fk.py tests/test_gpu_parity.py tests/test_gpu_dropout.py tests/test_gpu_fused.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_train_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_train_tests.log; grep -E "^FAILED" gpurun_out/r5_train_tests.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python tools/train_bench.py --modes kernel --steps 50 --warmup 10 --warmup-s 1 > gpurun_out/r5_train_a.log 2>&1 || { tail -5 gpurun_out/r5_train_a.log; exit 4; }
echo "default adam: $(grep -i "kernel" gpurun_out/r5_train_a.log | tail -1)"
