#!/bin/bash
# Memory-pipeline counters of the fp32 layer kernel at config 2 (kbench fk_fused64 = the shipping
# two-workgroup walk), one rocprofv3 --pmc pass per counter group; the counter list of the box first.
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/prof_r6_fkpmc
mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
A="tools/kbench.py --only fk_fused64 --rounds 3"
i=0
while read -r G; do
  [ -z "$G" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G -T --output-format csv -d "$OUT/p$i" -o run -- python3 $A > "$OUT/p$i.log" 2>&1 || echo "pass $i ($G) failed rc=$?"
done <<'GROUPS'
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUFFER_WAVEFRONTS_sum
TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_WRITE_TAGCONFLICT_STALL_CYCLES_sum
TCC_HIT_sum TCC_MISS_sum
TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum
GRBM_GUI_ACTIVE GRBM_COUNT
GROUPS
python3 tools/pmc_summary.py "$OUT" 2>/dev/null | sed -n '/update_fk_kernel/,/== /p'
echo "fk pmc done"
