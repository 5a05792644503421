#!/bin/bash
# the page-locked slot ring feed: loader tests, then feed_diag with / without the ring, /dev/shm size
set -uo pipefail
mkdir -p gpurun_out
df -h /dev/shm | tail -1
timeout -k 10 300 python -u -m pytest tests/test_gpu_loader.py -x -v --timeout 120 --timeout-method thread > gpurun_out/c11_tests.log 2>&1 || { tail -30 gpurun_out/c11_tests.log; exit 2; }
tail -1 gpurun_out/c11_tests.log
for cfg in "8 3" "14 3" "14 0"; do
  set -- $cfg
  timeout -k 10 300 python tools/feed_diag.py --workers $1 --ring-slots $2 > gpurun_out/feed_ring_$1_$2.txt 2>&1 || { tail -30 gpurun_out/feed_ring_$1_$2.txt; exit 3; }
  tail -1 gpurun_out/feed_ring_$1_$2.txt
done
