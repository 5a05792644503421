#!/bin/bash
# kernel-level A/B of the amax atomics change (see tools/r5_amax.sh)
set -uo pipefail
mkdir -p gpurun_out
for r in 1 2; do for L in "" variant:ab0; do
  echo "== lib '$L'"; NT_LIB=$L timeout -k 10 300 python tools/kbench.py --only init,fk_fused64,fk_fused --rounds 7 2>&1 | tail -6 || exit 5
done; done
