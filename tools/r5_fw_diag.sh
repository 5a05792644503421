#!/bin/bash
# fw vs fk diagnostics: mismatch map, stamp build, two PMC passes over the A/B tool (both kernels).
set -uo pipefail
mkdir -p gpurun_out/pmc_fw
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
[ -n "${MAIN:-}" ] && { timeout -k 10 180 python -u tools/fw_check.py --mols 4096 --rev nodes > gpurun_out/fwd_q4k.log 2>&1; cat gpurun_out/fwd_q4k.log; }
[ -n "${STAMP:-}" ] && NT_LIB=variant:fwstamp timeout -k 10 180 python -u tools/fw_check.py --mols 4096 --rev nodes --rounds 2 > gpurun_out/fwd_stamp.log 2>&1; grep -E "stamps|fw128|fk128" gpurun_out/fwd_stamp.log; true
for b in 835 3907 1859 2883; do
  NT_LIB=variant:fwabl NT_FK_RTABL=$b timeout -k 10 120 python -u tools/fw_check.py --mols 4096 --rev nodes --rounds 3 > gpurun_out/fwd_abl$b.log 2>&1; echo "abl $b: $(grep -E 'fw128|fk128' gpurun_out/fwd_abl$b.log | tr '\n' ' ')"
done

[ -n "${PMC:-}" ] && timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -T --output-format csv -d gpurun_out/pmc_fw/p1 -o run -- python3 tools/fw_check.py --rounds 1 > gpurun_out/pmc_fw/p1.log 2>&1 || { tail -5 gpurun_out/pmc_fw/p1.log; exit 3; }
[ -n "${PMC:-}" ] && timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -T --output-format csv -d gpurun_out/pmc_fw/p2 -o run -- python3 tools/fw_check.py --rounds 1 > gpurun_out/pmc_fw/p2.log 2>&1 || { tail -5 gpurun_out/pmc_fw/p2.log; exit 4; }
[ -n "${PMC:-}" ] && timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE -T --output-format csv -d gpurun_out/pmc_fw/p3 -o run -- python3 tools/fw_check.py --rounds 1 > gpurun_out/pmc_fw/p3.log 2>&1 || { tail -5 gpurun_out/pmc_fw/p3.log; exit 5; }
python3 tools/pmc_summary.py gpurun_out/pmc_fw 2>/dev/null | grep -A24 "update_f[kw]_kernel" || true
echo diag done
