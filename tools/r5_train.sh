#!/bin/bash
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_parity.py tests/test_gpu_fk.py tests/test_gpu_dropout.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_train_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_train_tests.log; grep -E "^FAILED" gpurun_out/r5_train_tests.log | head; [ $rc -eq 0 ] || exit $rc
for F in 1 0; do
  NT_FUSED_DA=$F timeout -k 10 240 python tools/train_bench.py --modes kernel --steps 50 --warmup 10 --warmup-s 1 > gpurun_out/r5_train_$F.log 2>&1 || { tail -5 gpurun_out/r5_train_$F.log; exit 4; }
  echo "fused dA=$F: $(grep -i "kernel" gpurun_out/r5_train_$F.log | tail -2 | tr '\n' ' ')"
done
