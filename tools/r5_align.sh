#!/bin/bash
# Row pitch A/B: 32-byte multiples (h = 300 -> 304, the default) against 128-byte L2 lines (-> 320)
set -uo pipefail
mkdir -p gpurun_out
for r in 1 2 3; do for A in 8 32; do
  NT_ROW_ALIGN=$A timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-embedded --no-training > gpurun_out/r5_align.log 2>&1 || { tail -5 gpurun_out/r5_align.log; exit 5; }
  echo "align $A: $(tail -1 gpurun_out/r5_align.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["secondary"]["polymer-16"]; print(round(d["ms_per_step"]*1e3,1), "us/step", round(d["roofline"]["launch_us"],1), "us/launch | polymer", round(s["ms_per_step"]*1e3,1), "us/step", round(s["roofline"]["launch_us"],1))')"
done; done
