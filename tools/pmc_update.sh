#!/bin/bash
# PMC counters of the update-kernel variants (one rocprofv3 pass per counter group).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TAG=${1:-pmc}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
ARGS="--only ${ONLY:-update,update_glds} --rounds 1 $*"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -T --output-format csv -d "$OUT/sq" -o run -- python3 tools/kbench.py $ARGS > "$OUT/sq.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -T --output-format csv -d "$OUT/inst" -o run -- python3 tools/kbench.py $ARGS > "$OUT/inst.log" 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace" -o run -- python3 tools/kbench.py $ARGS > "$OUT/trace.log" 2>&1
echo done
