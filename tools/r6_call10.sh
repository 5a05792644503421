#!/bin/bash
# host-feed breakdown (tools/feed_diag.py): DataLoader pin thread vs a 4-thread pin pool, 8 / 14 workers
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_loader.py -x -v --timeout 120 --timeout-method thread > gpurun_out/c10_tests.log 2>&1 || { tail -30 gpurun_out/c10_tests.log; exit 2; }
tail -1 gpurun_out/c10_tests.log
for cfg in "8 0" "8 4" "14 0" "14 4"; do
  set -- $cfg
  timeout -k 10 300 python tools/feed_diag.py --workers $1 --pin-threads $2 > gpurun_out/feed_diag_$1_$2.txt 2>&1 || { tail -30 gpurun_out/feed_diag_$1_$2.txt; exit 3; }
  tail -1 gpurun_out/feed_diag_$1_$2.txt
done
