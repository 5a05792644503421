#!/bin/bash
# hub-graph init: the chunked init (default) against the wave-per-node init (NT_HUB_INIT=wave)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for r in 1 2; do for M in chunked wave; do
  NT_HUB_INIT=$M timeout -k 10 300 python bench.py --workload polymer-16 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r5_hi.log 2>&1 || { tail -5 gpurun_out/r5_hi.log; exit 5; }
  echo "$M: $(tail -1 gpurun_out/r5_hi.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step")')"
done; done
