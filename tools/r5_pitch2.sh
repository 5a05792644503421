#!/bin/bash
# row pitch at HBM scale (qm9-32k: H = 745 MB > the 256 MB MALL): h = 300 against h = 304
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for H in 300 304 300 304; do
  echo "h=$H"
  timeout -k 10 180 python tools/kbench.py --mols 32768 --h $H --only init,fk_fused --rounds 3 > gpurun_out/kb_pitch.log 2>&1 || { tail -5 gpurun_out/kb_pitch.log; exit 3; }
  grep median gpurun_out/kb_pitch.log
done
