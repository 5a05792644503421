#!/bin/bash
# training step with padded forward states (default) against dense rows (NT_ROW_PAD=0), same box
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for r in 1 2 3; do for P in 1 0; do
  NT_ROW_PAD=$P timeout -k 10 240 python tools/train_bench.py --modes kernel --steps 50 --warmup 10 --warmup-s 1 > gpurun_out/r5_tpab.log 2>&1 || { tail -5 gpurun_out/r5_tpab.log; exit 4; }
  echo "pad=$P: $(grep -i "kernel" gpurun_out/r5_tpab.log | tail -1)"
done; done
