#!/bin/bash
# End-of-round evidence: full GPU suite, smoke, profile package (trace + FETCH/WRITE/SQ PMC passes +
# a bench line with measured traffic) for the judged workloads, the default bench line, and the
# config-4 workload on one GPU.  Every step has its own time limit; stops at the first failure.
set -uo pipefail
TAG=${1:-r2c}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -20 gpurun_out/gpu_tests.log; exit 2; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 3; }
tools/profile_round.sh "$TAG" qm9-4096 qm9-32k zinc-4096-bf16 || exit 4
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 5; }
tail -1 gpurun_out/bench_default.log | cut -c1-300
timeout -k 10 400 python bench.py --workload qm9-1m-sharded --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_config4.log 2>&1 || { tail -20 gpurun_out/bench_config4.log; exit 6; }
tail -1 gpurun_out/bench_config4.log | cut -c1-300
timeout -k 10 200 python tools/train_bench.py > gpurun_out/train.log 2>&1 || exit 7
tail -4 gpurun_out/train.log
