#!/bin/bash
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for L in "" "variant:im0"; do
  NT_LIB=$L timeout -k 10 120 python tools/kbench.py --only init,fk_fused64 --rounds 5 > gpurun_out/kb_init_$L.log 2>&1; echo "lib '$L':"; grep median gpurun_out/kb_init_$L.log
done
