#!/bin/bash
# W-fragment cache-policy A/B (variants waux1 = sc0, waux2 = nt): kbench of the layer kernel and bench lines
set -uo pipefail
mkdir -p gpurun_out
for r in 1 2; do for L in "" variant:waux1 variant:waux2; do
  echo "== lib '$L'"; NT_LIB=$L timeout -k 10 300 python tools/kbench.py --only fk_fused64 --rounds 7 2>&1 | grep -E "median" || exit 5
done; done
for r in 1 2; do for L in "" variant:waux1 variant:waux2; do
  NT_LIB=$L timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r6_c7.log 2>&1 || { tail -5 gpurun_out/r6_c7.log; exit 5; }
  echo "lib '$L': $(tail -1 gpurun_out/r6_c7.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["ms_per_step"]*1e3,1), "us/step", round(r["launch_us"],1), "us/launch")')"
done; done
