#!/bin/bash
# ring feed (collate into slots) with the background H2D thread vs inline
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_loader.py -x -v --timeout 120 --timeout-method thread > gpurun_out/c13_tests.log 2>&1 || { tail -30 gpurun_out/c13_tests.log; exit 2; }
tail -1 gpurun_out/c13_tests.log
for opt in "" "--inline"; do
  timeout -k 10 300 python tools/feed_diag.py --workers 14 $opt > gpurun_out/feed13$opt.txt 2>&1 || { tail -30 gpurun_out/feed13$opt.txt; exit 3; }
  tail -1 gpurun_out/feed13$opt.txt
done
