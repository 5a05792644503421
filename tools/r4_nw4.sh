#!/bin/bash
# A/B of the two-workgroups-per-CU fp32 layer kernel (NT_FK_NW=4): parity under it, kbench against
# the shipping walk, the config-2 bench line both ways.
set -uo pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
NT_FK_NW=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_fk.py tests/test_gpu_parity.py tests/test_gpu_fused.py -q --timeout 120 --timeout-method thread > gpurun_out/nw4_tests.log 2>&1
tail -2 gpurun_out/nw4_tests.log; grep -E "^FAILED" gpurun_out/nw4_tests.log | head -12
timeout -k 10 180 python tools/kbench.py --only fk_fused,fk_fused64 --rounds 5 > gpurun_out/nw4_kb0.log 2>&1 || exit 3
NT_FK_NW=4 timeout -k 10 180 python tools/kbench.py --only fk_fused64 --rounds 5 > gpurun_out/nw4_kb4.log 2>&1 || exit 3
grep median gpurun_out/nw4_kb0.log; echo "NW4: $(grep median gpurun_out/nw4_kb4.log)"
for v in 8 4; do
  NT_FK_NW=$v timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/nw4_b$v.log 2>&1 || exit 4
  echo "NW$v: $(tail -1 gpurun_out/nw4_b$v.log | grep -o '"ms_per_step": [0-9.]*\|"launch_us": [0-9.]*' | tr '\n' ' ')"
done
