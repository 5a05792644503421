#!/bin/bash
# loader / integration tests, the host-feed sweep (tools/feed_bench.py), the config-2 profile package
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_loader.py tests/test_gpu_integration.py -x -v --timeout 120 --timeout-method thread > gpurun_out/c9_tests.log 2>&1 || { tail -30 gpurun_out/c9_tests.log; exit 2; }
tail -2 gpurun_out/c9_tests.log
timeout -k 10 400 python tools/feed_bench.py --workers 8,14 --profile > gpurun_out/feed_bench.txt 2>&1 || { tail -30 gpurun_out/feed_bench.txt; exit 3; }
head -60 gpurun_out/feed_bench.txt
bash tools/profile_round.sh r6 qm9-4096 || exit 4
