#!/bin/bash
# Round-5 A/B of update_fw_kernel against update_fk_kernel (bit-exact + timings), several batches.
set -uo pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 python -u tools/fw_check.py --mols 4096 --rev nodes > gpurun_out/fw_q4k.log 2>&1; rc=$?; cat gpurun_out/fw_q4k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u tools/fw_check.py --mols 4096 --rev edges --agg identity > gpurun_out/fw_q4k_e.log 2>&1; rc=$?; cat gpurun_out/fw_q4k_e.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/fw_check.py --mols 32768 --rev nodes > gpurun_out/fw_q32k.log 2>&1; rc=$?; cat gpurun_out/fw_q32k.log; [ $rc -eq 0 ] || exit $rc
