#!/bin/bash
# A/B: bf16 layer on the two-workgroup 64-row fk walk (NT_BF16_KERNEL=fk4) against the 64-row bf16 kernel.
set -uo pipefail
mkdir -p gpurun_out
NT_BF16_KERNEL=fk4 timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_bf16_backward.py -q --timeout 120 --timeout-method thread > gpurun_out/fkb4_tests.log 2>&1
tail -1 gpurun_out/fkb4_tests.log; grep -E "^FAILED" gpurun_out/fkb4_tests.log | head -5
for r in 1 2; do for v in default fk4; do
  if [ $v = default ]; then K=""; else K=$v; fi
  NT_BF16_KERNEL=$K timeout -k 10 300 python bench.py --workload zinc-4096-bf16 --steps 30 --warmup 6 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/fkb_${v}.log 2>&1 || { tail -3 gpurun_out/fkb_${v}.log; exit 4; }
  echo "zinc $v r$r: $(tail -1 gpurun_out/fkb_${v}.log | grep -o '"ms_per_step": [0-9.]*\|"launch_us": [0-9.]*' | tr '\n' ' ')"
done; done
