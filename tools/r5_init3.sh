#!/bin/bash
# flat XCD-aware init against the wave-per-node init (variant if0) and the flat init without the
# XCD remap (variant ix0): parity tests, kbench, bench
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_layerwise.py tests/test_gpu_numerics.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_init_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_init_tests.log; grep -E "^FAILED" gpurun_out/r5_init_tests.log | head; [ $rc -eq 0 ] || exit $rc
for L in "" "variant:if0" "variant:ix0"; do echo "lib '$L':"; NT_LIB=$L timeout -k 10 120 python tools/kbench.py --only init,init_noamax,add --rounds 5 | grep median || exit 4; done
for L in "" "variant:if0"; do
NT_LIB=$L timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r5_b.log 2>&1 || { tail -5 gpurun_out/r5_b.log; exit 5; }
echo "bench '$L': $(tail -1 gpurun_out/r5_b.log | grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"
done
