#!/bin/bash
# One GPU-box pass: the new-kernel tests first (FIRST, optional), the -m gpu parity suite, smoke(),
# the default bench line, the N=2 launcher rehearsal (REHEARSE=1), the training bench (TRAIN=1).
# Every GPU step has its own time limit; the script stops at the first failing step.
set -uo pipefail
mkdir -p gpurun_out
if [ -n "${FIRST:-}" ]; then
  timeout -k 10 400 python -u -m pytest $FIRST -x -v --timeout 120 --timeout-method thread > gpurun_out/first_tests.log 2>&1
  rc=$?; tail -4 gpurun_out/first_tests.log; grep -E "FAILED|ERROR" gpurun_out/first_tests.log | head -20
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log; grep -E "FAILED|ERROR" gpurun_out/gpu_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 3; }
cat gpurun_out/smoke.log
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 4; }
tail -1 gpurun_out/bench.log | cut -c1-1500
if [ -n "${REHEARSE:-}" ]; then
  timeout -k 10 300 python bench.py --gpus 2 --same-device --dist-backend gloo --steps 10 --warmup 3 --no-secondary \
    --no-embedded --cpu-seconds 2 > gpurun_out/rehearse2.log 2>&1 || { tail -20 gpurun_out/rehearse2.log; exit 5; }
  tail -1 gpurun_out/rehearse2.log | cut -c1-600
fi
if [ -n "${TRAIN:-}" ]; then
  timeout -k 10 200 python tools/train_bench.py > gpurun_out/train.log 2>&1 || { tail -20 gpurun_out/train.log; exit 6; }
  tail -5 gpurun_out/train.log
fi
exit $rc
