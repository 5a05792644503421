#!/bin/bash
# Generic A/B of the shipping library against variant ab0 (built with make VARIANT=ab0 EXTRA=...):
# the GPU parity tests on the shipping library, kbench of KB kernels, then bench.py lines.
# Usage: KB=init TESTS="tests/test_gpu_parity.py ..." bash tools/r5_ab.sh
set -uo pipefail
mkdir -p gpurun_out
TESTS=${TESTS:-"tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_hubs.py"}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_ab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_ab_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/r5_ab_tests.log | head; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for L in "" variant:ab0; do
  echo "== lib '$L'"; NT_LIB=$L timeout -k 10 300 python tools/kbench.py --only ${KB:-init} --rounds 7 2>&1 | grep -E "median" || exit 5
done; done
for r in 1 2 3; do for L in "" variant:ab0; do
  NT_LIB=$L timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r5_ab.log 2>&1 || { tail -5 gpurun_out/r5_ab.log; exit 5; }
  echo "lib '$L': $(tail -1 gpurun_out/r5_ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,1), "us/step", round(d["roofline"]["launch_us"],1), "us/launch")')"
done; done
