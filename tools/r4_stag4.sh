#!/bin/bash
# A/B: start delay of the second workgroup half in the two-workgroup walk (NT_FK_STAGGER x 8k cycles).
set -uo pipefail
mkdir -p gpurun_out
for r in 1 2; do for v in 0 2 4 6; do
  NT_FK_STAGGER=$v timeout -k 10 300 python bench.py --steps 40 --warmup 8 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/st4_$v.log 2>&1 || exit 4
  echo "stagger $v r$r: $(tail -1 gpurun_out/st4_$v.log | grep -o '"ms_per_step": [0-9.]*\|"launch_us": [0-9.]*' | tr '\n' ' ')"
done; done
