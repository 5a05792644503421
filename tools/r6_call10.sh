#!/bin/bash
# host-feed breakdown (tools/feed_diag.py) at 8 and 14 workers
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/feed_diag.py --workers 8 > gpurun_out/feed_diag8.txt 2>&1 || { tail -30 gpurun_out/feed_diag8.txt; exit 2; }
tail -1 gpurun_out/feed_diag8.txt
timeout -k 10 300 python tools/feed_diag.py --workers 14 > gpurun_out/feed_diag14.txt 2>&1 || { tail -30 gpurun_out/feed_diag14.txt; exit 3; }
tail -1 gpurun_out/feed_diag14.txt
