#!/bin/bash
# NT_FK_NW A/B on the bench lines, alternating, two rounds per workload.
set -uo pipefail
mkdir -p gpurun_out
for W in ${WLS:-qm9-4096 polymer-16 qm9-32k}; do
  for r in 1 2; do for v in 8 4; do
    NT_FK_NW=$v timeout -k 10 300 python bench.py --workload $W --steps 40 --warmup 8 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/nwb_${W}_${v}.log 2>&1 || { tail -3 gpurun_out/nwb_${W}_${v}.log; exit 4; }
    echo "$W NW$v r$r: $(tail -1 gpurun_out/nwb_${W}_${v}.log | grep -o '"ms_per_step": [0-9.]*\|"launch_us": [0-9.]*' | tr '\n' ' ')"
  done; done
done
