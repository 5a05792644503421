#!/bin/bash
# A/B of an fk-kernel experiment knob (env VAR over VALUES) on the config-2 bench line, a fresh
# process per value, two rounds.  Usage: VAR=NT_FK_NTSTORE VALUES="0 1 2 3" bash tools/fk_ab.sh
set -uo pipefail
mkdir -p gpurun_out
for R in 1 2; do
  for X in $VALUES; do
    env $VAR=$X timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary --no-embedded --no-training ${BENCH_ARGS:-} > gpurun_out/ab_${X}_$R.log 2>&1 || { tail -20 gpurun_out/ab_${X}_$R.log; exit 4; }
    echo "$VAR=$X round $R: $(tail -1 gpurun_out/ab_${X}_$R.log | grep -o '"ms_per_step": [0-9.]*\|"launch_us": [0-9.]*' | tr '\n' ' ')"
  done
done
