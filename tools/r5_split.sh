#!/bin/bash
# hub-graph init: fused chunked init (padded / dense rows) against plain init + chunked reduce (dense)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for r in 1 2; do for E in "NT_ROW_PAD=1" "NT_ROW_PAD=0" "NT_INIT_SPLIT=1"; do
  env $E timeout -k 10 300 python bench.py --workload polymer-16 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r5_split.log 2>&1 || { tail -5 gpurun_out/r5_split.log; exit 5; }
  echo "$E: $(tail -1 gpurun_out/r5_split.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step", round(d["roofline"]["launch_us"],1), "us/launch")')"
done; done
