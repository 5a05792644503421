#!/bin/bash
# ring feed with slice batches and no pin thread; profile of a fresh-batch forward's host work
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_loader.py -x -v --timeout 120 --timeout-method thread > gpurun_out/c12_tests.log 2>&1 || { tail -30 gpurun_out/c12_tests.log; exit 2; }
tail -1 gpurun_out/c12_tests.log
timeout -k 10 300 python tools/feed_diag.py --workers 14 --ring-slots 3 --profile > gpurun_out/feed_ring_prof.txt 2>&1 || { tail -30 gpurun_out/feed_ring_prof.txt; exit 3; }
cat gpurun_out/feed_ring_prof.txt
timeout -k 10 300 python tools/feed_diag.py --workers 12 --ring-slots 3 > gpurun_out/feed_ring_12.txt 2>&1 || { tail -30 gpurun_out/feed_ring_12.txt; exit 4; }
tail -1 gpurun_out/feed_ring_12.txt
