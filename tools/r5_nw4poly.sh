#!/bin/bash
# polymer-16 with 128-byte hub rows: 128-row walk (default, E > NW4_MAX_EDGES) vs the 64-row
# two-workgroup walk (NT_NW4_MAX_EDGES raised past polymer's 456k edges)
set -uo pipefail
mkdir -p gpurun_out
for r in 1 2 3; do for M in 131072 1000000; do
  NT_NW4_MAX_EDGES=$M timeout -k 10 300 python bench.py --workload polymer-16 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r5_nw4poly.log 2>&1 || { tail -5 gpurun_out/r5_nw4poly.log; exit 5; }
  echo "max_edges $M: $(tail -1 gpurun_out/r5_nw4poly.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,1), "us/step", round(d["roofline"]["launch_us"],1), "us/launch")')"
done; done
