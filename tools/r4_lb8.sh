#!/bin/bash
# A/B: the bias in LDS for the 8-wave 128-row fp32 walk (variant lb8) on the workloads that use it.
set -uo pipefail
mkdir -p gpurun_out
NT_LIB=variant:lb8 timeout -k 10 300 python -u -m pytest tests/test_gpu_fk.py -q --timeout 120 --timeout-method thread > gpurun_out/lb8_tests.log 2>&1 || { tail -5 gpurun_out/lb8_tests.log; exit 3; }
tail -1 gpurun_out/lb8_tests.log
for W in polymer-16 qm9-32k; do for r in 1 2; do for v in base lb8; do
  if [ $v = base ]; then L=""; else L=variant:$v; fi
  NT_LIB=$L timeout -k 10 300 python bench.py --workload $W --steps 30 --warmup 6 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/lb_${W}_${v}.log 2>&1 || exit 4
  echo "$W $v r$r: $(tail -1 gpurun_out/lb_${W}_${v}.log | grep -o '"ms_per_step": [0-9.]*\|"launch_us": [0-9.]*' | tr '\n' ' ')"
done; done; done
