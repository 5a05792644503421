#!/bin/bash
# Instruction-mix / wait counters of the fp32 layer kernel at config 2 (two --pmc passes of <= 8 SQ
# counters each, no trace domains), for locating what the update_fk K loop and epilogue wait on.
set -uo pipefail
mkdir -p gpurun_out/pmc_fk
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-embedded --no-training"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -T --output-format csv -d gpurun_out/pmc_fk/p1 -o run -- python3 bench.py $ARGS > gpurun_out/pmc_fk/p1.log 2>&1 || { tail -5 gpurun_out/pmc_fk/p1.log; exit 3; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -T --output-format csv -d gpurun_out/pmc_fk/p2 -o run -- python3 bench.py $ARGS > gpurun_out/pmc_fk/p2.log 2>&1 || { tail -5 gpurun_out/pmc_fk/p2.log; exit 4; }
python3 tools/pmc_summary.py gpurun_out/pmc_fk 2>/dev/null | grep -A12 update_fk || true
echo pmc done
