#!/bin/bash
# GraphFeeder (DataLoader-free ring feed): loader tests, feed_diag at 14 / 12 workers, the bench's pipelined leg
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_loader.py -x -v --timeout 120 --timeout-method thread > gpurun_out/c14_tests.log 2>&1 || { tail -30 gpurun_out/c14_tests.log; exit 2; }
tail -1 gpurun_out/c14_tests.log
for W in 14 12; do
  timeout -k 10 300 python tools/feed_diag.py --workers $W > gpurun_out/feed14_$W.txt 2>&1 || { tail -30 gpurun_out/feed14_$W.txt; exit 3; }
  tail -1 gpurun_out/feed14_$W.txt
done
timeout -k 10 300 python tools/feed_bench.py --workers 14 > gpurun_out/feed_bench14.txt 2>&1 || { tail -30 gpurun_out/feed_bench14.txt; exit 4; }
tail -3 gpurun_out/feed_bench14.txt
