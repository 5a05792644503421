#!/bin/bash
# A/B of the row-padded intermediates (NT_ROW_PAD=1, default) against dense rows, alternating runs
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for r in 1 2 3; do for P in 1 0; do
  NT_ROW_PAD=$P timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r5_pad.log 2>&1 || { tail -5 gpurun_out/r5_pad.log; exit 5; }
  echo "pad=$P: $(tail -1 gpurun_out/r5_pad.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,1), "us/step", round(d["roofline"]["launch_us"],1), "us/launch")')"
done; done
