#!/bin/bash
# A/B of the 64-row tile plans' balance (NT_PLAN_SLOTS64 = 256 CUs vs 512 = two workgroups per CU):
# config 2 and config 3 bench lines, alternating, then config-2 training steps.
set -uo pipefail
mkdir -p gpurun_out
for W in qm9-4096 zinc-4096-bf16; do for r in 1 2 3; do for S in 256 512; do
  NT_PLAN_SLOTS64=$S timeout -k 10 300 python bench.py --workload $W --steps 50 --warmup 10 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r6_slots.log 2>&1 || { tail -5 gpurun_out/r6_slots.log; exit 5; }
  echo "$W slots $S: $(tail -1 gpurun_out/r6_slots.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["ms_per_step"]*1e3,1), "us/step", round(r["launch_us"],1), "us/launch")')"
done; done; done
for r in 1 2; do for S in 256 512; do
  echo "train slots $S: $(NT_PLAN_SLOTS64=$S timeout -k 10 300 python tools/train_bench.py --json --modes kernel --steps 50 --warmup 10 --warmup-s 1 2>/dev/null | tail -1 | cut -c1-200)"
done; done
