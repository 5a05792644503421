#!/bin/bash
# segment_reduce_block (contiguous segments: the readouts) vs the row-piece wave kernel (variant seg0):
# the parity tests on the shipping build, then kbench of the Sum readout and bench lines, alternating.
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_readout.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/seg_tests.log 2>&1
rc=$?; tail -2 gpurun_out/seg_tests.log; grep -E "^FAILED|Error" gpurun_out/seg_tests.log | head; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for L in "" variant:seg0; do
  echo "== lib '$L'"; NT_LIB=$L timeout -k 10 300 python tools/kbench.py --only readout --rounds 9 2>&1 | grep -E "median" || exit 5
done; done
for r in 1 2; do for L in "" variant:seg0; do
  NT_LIB=$L timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/seg_ab.log 2>&1 || { tail -5 gpurun_out/seg_ab.log; exit 5; }
  echo "lib '$L': $(tail -1 gpurun_out/seg_ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["ms_per_step"]*1e3,1), "us/step", round(r["launch_us"],1), "us/launch")')"
done; done
