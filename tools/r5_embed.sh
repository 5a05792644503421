#!/bin/bash
# embedded encoder with padded rows: tests, then the bench line (embedded leg included)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_embed.py tests/test_gpu_fused.py tests/test_gpu_graphs.py tests/test_gpu_integration.py tests/test_gpu_loader.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_embed_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_embed_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/r5_embed_tests.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary --no-training > gpurun_out/r5_embed_b.log 2>&1 || { tail -5 gpurun_out/r5_embed_b.log; exit 5; }
tail -1 gpurun_out/r5_embed_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("embedded"))'
