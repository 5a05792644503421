#!/bin/bash
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for r in 1 2; do for L in "" variant:w8b16 variant:w16b16 variant:w16b4; do
  NT_LIB=$L timeout -k 10 120 python tools/hub_bench.py > gpurun_out/hub.log 2>&1 || { tail -5 gpurun_out/hub.log; exit 3; }
  tail -1 gpurun_out/hub.log
done; done
