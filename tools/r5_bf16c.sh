#!/bin/bash
# bf16 layer kernel A/B: the 64-row bf16 kernel (default), fk4 (8 column tiles per wave), fk4c (4 column
# tiles per wave, 256-column chunks; 2 or 3 workgroups per CU); bf16 parity tests under fk4c first
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
NT_BF16_KERNEL=fk4c timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_bf16_backward.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_bf16c_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_bf16c_tests.log; grep -E "^FAILED" gpurun_out/r5_bf16c_tests.log | head; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for K in "" fk4 fk4c fk4c3; do
  KK=$K; W=2; [ "$K" = fk4c3 ] && { KK=fk4c; W=3; }
  NT_FKB_WG=$W NT_BF16_KERNEL=$KK timeout -k 10 120 python tools/bf16_kb.py > gpurun_out/bf16_kb.log 2>&1 || { tail -5 gpurun_out/bf16_kb.log; exit 3; }
  echo "$K: $(tail -1 gpurun_out/bf16_kb.log)"
done; done
