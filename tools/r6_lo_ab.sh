#!/bin/bash
# A/B of the shipping library (scaled low part + 8-row readout batches) against lo0 (the round-5 split
# and 4-row readout batches) and prio (static priority for the second workgroup per CU): kbench of the
# layer kernel and the Sum readout, then default bench lines, alternating.
set -uo pipefail
mkdir -p gpurun_out
for r in 1 2; do for L in "" variant:lo0 variant:prio; do
  echo "== lib '$L'"; NT_LIB=$L timeout -k 10 300 python tools/kbench.py --only fk_fused64,readout --rounds 7 2>&1 | grep -E "median" || exit 5
done; done
for r in 1 2 3; do for L in "" variant:lo0 variant:prio; do
  NT_LIB=$L timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r6_ab.log 2>&1 || { tail -5 gpurun_out/r6_ab.log; exit 5; }
  echo "lib '$L': $(tail -1 gpurun_out/r6_ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["ms_per_step"]*1e3,1), "us/step", round(r["launch_us"],1), "us/launch frac", round(r["frac"],3))')"
done; done
