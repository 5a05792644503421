#!/bin/bash
# A/B of shipping-source variant builds (make VARIANT=<v> EXTRA=...) on the fp32 layer kernel alone
# (tools/kbench.py, config-2 batch), a fresh process per variant, two rounds.
# Usage: VARIANTS="base mb" [ONLY=fk_fused,init] bash tools/r4_ab.sh
set -uo pipefail
mkdir -p gpurun_out
for R in 1 2; do
  for V in $VARIANTS; do
    if [ "$V" = base ]; then L=""; else L="variant:$V"; fi
    NT_LIB=$L timeout -k 10 200 python tools/kbench.py --only ${ONLY:-fk_fused,init} --rounds 5 > gpurun_out/ab_${V}_$R.log 2>&1 || { tail -20 gpurun_out/ab_${V}_$R.log; exit 4; }
    echo "$V round $R: $(grep -E 'median' gpurun_out/ab_${V}_$R.log | tr -s ' ' | tr '\n' '|')"
  done
done
