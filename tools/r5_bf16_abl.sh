#!/bin/bash
# bf16 layer kernel phase ablations (BF_ABL variant builds; results wrong by construction)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for L in "" variant:ba1 variant:ba2 variant:ba12 variant:ba16 variant:ba15 variant:ba28 ""; do
  NT_LIB=$L timeout -k 10 120 python tools/bf16_kb.py > gpurun_out/bf16_kb.log 2>&1 || { tail -5 gpurun_out/bf16_kb.log; exit 3; }
  tail -1 gpurun_out/bf16_kb.log
done
