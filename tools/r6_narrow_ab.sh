#!/bin/bash
# A/B of the narrow-front tile walk (VARIANT=narrow, FK_NARROW=1) against the shipping XCD-chunk walk:
# bit-identity of the block forward, the polymer / config-2 parity tests on the variant, then bench
# lines per workload, alternating.
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/bitcmp.py --save ship > gpurun_out/nar_bit.log 2>&1 || { tail -5 gpurun_out/nar_bit.log; exit 3; }
NT_LIB=variant:narrow timeout -k 10 300 python tools/bitcmp.py --save narrow >> gpurun_out/nar_bit.log 2>&1 || { tail -5 gpurun_out/nar_bit.log; exit 3; }
python tools/bitcmp.py --compare ship narrow | tail -6
NT_LIB=variant:narrow timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "polymer or config2 or hub or bf16" --timeout 300 --timeout-method thread > gpurun_out/nar_tests.log 2>&1
rc=$?; tail -2 gpurun_out/nar_tests.log; [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
for W in polymer-16 zinc-4096-bf16 qm9-32k qm9-4096; do for r in 1 2; do for L in "" variant:narrow; do
  NT_LIB=$L timeout -k 10 300 python bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/nar_ab.log 2>&1 || { tail -5 gpurun_out/nar_ab.log; exit 5; }
  echo "$W lib '$L': $(tail -1 gpurun_out/nar_ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["ms_per_step"]*1e3,1), "us/step", round(r["launch_us"],1), "us/launch frac", round(r["frac"],3))')"
done; done; done
