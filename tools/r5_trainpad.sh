#!/bin/bash
# padded training states: backward / hub / fused tests, then the training step (default Adam)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_bf16_backward.py tests/test_gpu_dropout.py tests/test_gpu_hubs.py tests/test_gpu_fused.py tests/test_gpu_layerwise.py tests/test_gpu_readout.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_tp_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_tp_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/r5_tp_tests.log | head; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 240 python tools/train_bench.py --modes kernel --steps 50 --warmup 10 --warmup-s 1 > gpurun_out/r5_tp_b.log 2>&1 || { tail -5 gpurun_out/r5_tp_b.log; exit 4; }
  echo "default adam: $(grep -i "kernel" gpurun_out/r5_tp_b.log | tail -1)"
done
