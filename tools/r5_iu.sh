#!/bin/bash
# rows in flight per lane of init_chunk_partial (polymer-16 forward)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for r in 1 2; do for L in "" variant:iu8 variant:iu2; do
  NT_LIB=$L timeout -k 10 300 python bench.py --workload polymer-16 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r5_iu.log 2>&1 || { tail -5 gpurun_out/r5_iu.log; exit 5; }
  echo "lib '$L': $(tail -1 gpurun_out/r5_iu.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step")')"
done; done
