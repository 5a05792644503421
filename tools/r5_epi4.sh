#!/bin/bash
set -uo pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 python -u tools/fw_check.py --mols 4096 --rev nodes > gpurun_out/e4_q4k.log 2>&1; cat gpurun_out/e4_q4k.log
NT_LIB=variant:epi3 timeout -k 10 180 python -u tools/fw_check.py --mols 4096 --rev nodes > gpurun_out/e4_q4k_old.log 2>&1; echo "== scan epilogue (old):"; grep "fk64\|fw128" gpurun_out/e4_q4k_old.log
timeout -k 10 180 python -u tools/fw_check.py --mols 4096 --rev edges --agg identity > gpurun_out/e4_q4k_e.log 2>&1; grep "bit-exact\|fk64" gpurun_out/e4_q4k_e.log
