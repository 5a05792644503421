#!/bin/bash
# PMC counters of the forward kernels under tools/kbench.py (one rocprofv3 pass per counter group,
# each under its own time limit).  Usage: ONLY=fk_fused bash tools/pmc_update.sh TAG [kbench args]
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TAG=${1:-pmc}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
ARGS="--only ${ONLY:-fk_fused} --rounds 1 $*"
run() {  # name, rocprofv3 args...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 "$@" -T --output-format csv -d "$OUT/$name" -o run -- python3 tools/kbench.py $ARGS \
    > "$OUT/$name.log" 2>&1 || { echo "pass $name failed: $?"; tail -5 "$OUT/$name.log"; exit 1; }
}
run trace --kernel-trace --stats
run sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run inst --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
echo done
