#!/bin/bash
# Round-4 iteration pass on the GPU box: named GPU tests (optional), then the config-2 bench line
# (and optionally the polymer-16 / zinc lines) without the slow legs, then a kernel-trace profile.
# Usage: TESTS="tests/a.py" [KEXPR=..] [WL="qm9-4096 polymer-16"] [PROF=1] bash tools/r4_iter.sh
set -uo pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -k "${KEXPR:-}" -x -q --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/iter_tests.log; grep -E "FAILED|ERROR|Error" gpurun_out/iter_tests.log | head -20
  [ $rc -eq 0 ] || exit $rc
fi
for W in ${WL:-qm9-4096}; do
  timeout -k 10 300 python bench.py --workload $W --steps 50 --warmup 10 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/bench_$W.log 2>&1 || { tail -20 gpurun_out/bench_$W.log; exit 4; }
  echo "$W: $(tail -1 gpurun_out/bench_$W.log | grep -o '"ms_per_step": [0-9.]*\|"launch_us": [0-9.]*\|"value": [0-9.e+]*' | tr '\n' ' ')"
done
if [ -n "${PROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_iter -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/prof_iter.log 2>&1 || { tail -20 gpurun_out/prof_iter.log; exit 7; }
  F=$(find gpurun_out/prof_iter -name "*kernel_stats.csv" | head -1); head -12 "$F" | cut -d, -f1-4
fi
exit 0
