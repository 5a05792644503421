#!/bin/bash
# A/B of the shipping library against variant $V (make VARIANT=$V EXTRA=...): bit-identity of the block
# forward, the GPU parity tests on the variant, kbench of $KB, then bench.py lines, alternating.
# Usage: V=ilv KB=fk_fused64 TESTS="tests/test_gpu_parity.py" bash tools/r6_ab.sh
set -uo pipefail
mkdir -p gpurun_out
V=${V:?variant}
KB=${KB:-fk_fused64}
timeout -k 10 300 python tools/bitcmp.py --save ship > gpurun_out/r6_bit.log 2>&1 || { tail -5 gpurun_out/r6_bit.log; exit 3; }
NT_LIB=variant:$V timeout -k 10 300 python tools/bitcmp.py --save $V >> gpurun_out/r6_bit.log 2>&1 || { tail -5 gpurun_out/r6_bit.log; exit 3; }
python tools/bitcmp.py --compare ship $V | tail -12
if [ -n "${TESTS:-}" ]; then
  NT_LIB=variant:$V timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_ab_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/r6_ab_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/r6_ab_tests.log | head; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do for L in "" variant:$V; do
  echo "== lib '$L'"; NT_LIB=$L timeout -k 10 300 python tools/kbench.py --only $KB --rounds 7 2>&1 | grep -E "median" || exit 5
done; done
for r in 1 2 3; do for L in "" variant:$V; do
  NT_LIB=$L timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r6_ab.log 2>&1 || { tail -5 gpurun_out/r6_ab.log; exit 5; }
  echo "lib '$L': $(tail -1 gpurun_out/r6_ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["ms_per_step"]*1e3,1), "us/step", round(r["launch_us"],1), "us/launch frac", round(r["frac"],3), r["kernel"])')"
done; done
