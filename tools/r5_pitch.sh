#!/bin/bash
# row pitch test: are dst-ordered row writes slower when rows are not whole 128-B lines (h = 300: 1200 B)?
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for H in 300 320 288 304; do
  echo "h=$H"
  timeout -k 10 180 python tools/kbench.py --h $H --only init,init_only,copy,fk_fused64 --rounds 5 > gpurun_out/kb_pitch.log 2>&1 || { tail -5 gpurun_out/kb_pitch.log; exit 3; }
  grep median gpurun_out/kb_pitch.log
done
