#!/bin/bash
# init kernel against the bandwidth ceilings of its traffic (copy / add of E-row tensors)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 180 python tools/kbench.py --only init,init_noamax,init_only,copy,add,fk_fused64 --rounds 5 > gpurun_out/kb_initbw.log 2>&1 || { tail -5 gpurun_out/kb_initbw.log; exit 3; }
cat gpurun_out/kb_initbw.log
