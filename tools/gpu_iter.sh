#!/bin/bash
# Iteration pass on the GPU box: the named tests, then the config-2 training step per weight-grad path
# (fresh process each), a kernel-stats profile of the training step, and the polymer-16 bench line.
# Usage: TESTS="tests/a.py tests/b.py" [KEXPR="expr"] bash tools/gpu_iter.sh
set -uo pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -k "${KEXPR:-}" -x -v --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/iter_tests.log; grep -E "FAILED|ERROR|Error" gpurun_out/iter_tests.log | head -20
  [ $rc -eq 0 ] || exit $rc
fi
for W in ${WGRADS:-kernel kernel6}; do
  NT_WGRAD=$W timeout -k 10 200 python tools/train_bench.py --modes kernel > gpurun_out/train_$W.log 2>&1 || { tail -20 gpurun_out/train_$W.log; exit 6; }
  echo "NT_WGRAD=$W"; tail -2 gpurun_out/train_$W.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_train -o run -- python3 tools/train_bench.py --modes kernel --steps 10 --warmup 3 > gpurun_out/prof_train.log 2>&1 || { tail -20 gpurun_out/prof_train.log; exit 7; }
F=$(find gpurun_out/prof_train -name "*kernel_stats.csv" | head -1); head -14 "$F" | cut -d, -f1-4
if [ -n "${POLY:-1}" ]; then
  timeout -k 10 300 python bench.py --workload polymer-16 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/bench_poly.log 2>&1 || { tail -20 gpurun_out/bench_poly.log; exit 4; }
  tail -1 gpurun_out/bench_poly.log | grep -o '"ms_per_step": [0-9.]*\|"launch_us": [0-9.]*\|"value": [0-9.e+]*' | head -3
fi
