#!/bin/bash
# Round-5 A/B of update_fw_kernel against update_fk_kernel (bit-exact + timings), several batches;
# then (TESTS=1) the fused-layer GPU tests with the fw walk selected everywhere it applies.
set -uo pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 python -u tools/fw_check.py --mols 4096 --rev nodes > gpurun_out/fw_q4k.log 2>&1; rc=$?; cat gpurun_out/fw_q4k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u tools/fw_check.py --mols 4096 --rev edges --agg identity > gpurun_out/fw_q4k_e.log 2>&1; rc=$?; cat gpurun_out/fw_q4k_e.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/fw_check.py --mols 32768 --rev nodes > gpurun_out/fw_q32k.log 2>&1; rc=$?; cat gpurun_out/fw_q32k.log; [ $rc -eq 0 ] || exit $rc
if [ -n "${TESTS:-}" ]; then
  NT_FK_FW=1 NT_FK_NW=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_fk.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_numerics.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fw_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/fw_tests.log; grep -E "^FAILED|Error" gpurun_out/fw_tests.log | head -20; [ $rc -eq 0 ] || exit $rc
fi
