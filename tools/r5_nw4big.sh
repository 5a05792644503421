#!/bin/bash
# 64-row two-workgroup walk against the 128-row walk on large graphs (padded rows)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for W in polymer-16 qm9-32k; do for M in 131072 100000000 131072 100000000; do
  NT_NW4_MAX_EDGES=$M timeout -k 10 300 python bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r5_nw4.log 2>&1 || { tail -5 gpurun_out/r5_nw4.log; exit 5; }
  echo "$W nw4max=$M: $(tail -1 gpurun_out/r5_nw4.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step", round(d["roofline"]["launch_us"],1), "us/launch")')"
done; done
