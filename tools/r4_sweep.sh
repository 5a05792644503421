#!/bin/bash
# Walk crossover: the fp32 layer's two-workgroup 64-row walk (NT_FK_NW=4 forces it) against the
# one-workgroup 128-row walk (NT_FK_NW=8) over batch sizes.
set -uo pipefail
mkdir -p gpurun_out
for W in ${WLS:-qm9-4096 qm9-8192 qm9-16k qm9-32k}; do for v in 8 4; do
  NT_FK_NW=$v timeout -k 10 300 python bench.py --workload $W --steps 30 --warmup 6 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/sw_${W}_${v}.log 2>&1 || exit 4
  echo "$W NW$v: $(tail -1 gpurun_out/sw_${W}_${v}.log | grep -o '"ms_per_step": [0-9.]*\|"launch_us": [0-9.]*\|"E_per_gpu": [0-9]*' | tr '\n' ' ')"
done; done
