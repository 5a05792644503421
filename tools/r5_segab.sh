#!/bin/bash
# segment_reduce_wave ragged last batch (default) vs batches of 4 then single rows (variant ab0):
# parity/backward tests, then bench lines with the training step
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_backward.py tests/test_gpu_readout.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_segab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_segab_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/r5_segab_tests.log | head; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for L in "" variant:ab0; do
  NT_LIB=$L timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary --no-embedded > gpurun_out/r5_segab.log 2>&1 || { tail -5 gpurun_out/r5_segab.log; exit 5; }
  echo "lib '$L': $(tail -1 gpurun_out/r5_segab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,1), "us/step", round(d["roofline"]["launch_us"],1), "us/launch | train", round(d["training"]["train_ms"],4), "ms")')"
done; done
