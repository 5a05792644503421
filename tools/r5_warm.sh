#!/bin/bash
# the driver's bench invocation (--steps 20 --warmup 5) against a longer one on the same box
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for r in 1 2; do for PW in "--prewarm-s 0" "--prewarm-s 1"; do for A in "20 5" "50 10"; do set -- $A
  timeout -k 10 300 python bench.py --steps $1 --warmup $2 $PW --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r5_w.log 2>&1 || { tail -5 gpurun_out/r5_w.log; exit 5; }
  echo "$PW steps $1 warmup $2: $(tail -1 gpurun_out/r5_w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,1), "us/step", round(d["roofline"]["launch_us"],1), "us/launch", d["value"])')"
done; done; done
