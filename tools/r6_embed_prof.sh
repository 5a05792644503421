#!/bin/bash
# Profile of the embedded encoder at config 2 (tools/embed_bench.py): kernel trace + separate PMC passes
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/prof_${TAG:-r6}_embed
mkdir -p "$OUT"
A="tools/embed_bench.py --steps 50 ${EARGS:-}"
timeout -k 10 300 python3 $A || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace" -o run -- python3 $A > "$OUT/trace.log" 2>&1 || exit 4
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$OUT/fetch" -o run -- python3 $A > "$OUT/fetch.log" 2>&1 || exit 5
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$OUT/write" -o run -- python3 $A > "$OUT/write.log" 2>&1 || exit 6
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE -T --output-format csv -d "$OUT/sq" -o run -- python3 $A > "$OUT/sq.log" 2>&1 || exit 7
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -T --output-format csv -d "$OUT/sq2" -o run -- python3 $A > "$OUT/sq2.log" 2>&1 || exit 8
python3 tools/pmc_summary.py "$OUT" 2>/dev/null | head -40 || true
echo "embed profile done"
