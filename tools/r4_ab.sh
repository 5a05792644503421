#!/bin/bash
# A/B of shipping-source variant builds (make VARIANT=<v> EXTRA=...) on the fp32 layer kernel alone
# (tools/kbench.py, config-2 batch), a fresh process per variant, two rounds.
# Usage: VARIANTS="base mb" [ONLY=fk_fused,init] bash tools/r4_ab.sh
set -uo pipefail
mkdir -p gpurun_out
if [ -n "${PARITY:-}" ]; then  # quick parity of each variant build (the wide fused fk tests)
  for V in $VARIANTS; do
    LIBV=${V%@*}; [ "$LIBV" != "$V" ] && continue
    if [ "$V" = base ]; then L=""; else L="variant:$V"; fi
    NT_LIB=$L timeout -k 10 300 python -u -m pytest ${PARITY_TESTS:-tests/test_gpu_fk.py -k "wide_plan or far_from"} -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_parity_$V.log 2>&1 || { echo "parity FAILED for $V"; tail -15 gpurun_out/ab_parity_$V.log; exit 5; }
    echo "parity $V: $(tail -1 gpurun_out/ab_parity_$V.log)"
  done
fi
for R in 1 2; do
  for V in $VARIANTS; do
    # V = <lib>[@<NT_FK_RTABL>]: a variant build, optionally with a runtime ablation mask
    LIBV=${V%@*}; AB=0; [ "$LIBV" != "$V" ] && AB=${V#*@}
    if [ "$LIBV" = base ]; then L=""; else L="variant:$LIBV"; fi
    NT_FK_RTABL=$AB NT_LIB=$L timeout -k 10 200 python tools/kbench.py --only ${ONLY:-fk_fused,init} --rounds 5 > gpurun_out/ab_${V}_$R.log 2>&1 || { tail -20 gpurun_out/ab_${V}_$R.log; exit 4; }
    echo "$V round $R: $(grep -E 'median' gpurun_out/ab_${V}_$R.log | tr -s ' ' | tr '\n' '|')"
  done
done
