#!/bin/bash
# Size-dependent row pitch: GPU tests over padded rows, then qm9-32k (HBM scale) at 32-B vs 128-B
# multiples (NT_ROW_ALIGN=8 / 32; the default picks 32 past NW4_MAX_EDGES) and the default bench line
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_hubs.py tests/test_gpu_config4.py tests/test_gpu_parity.py tests/test_gpu_embed.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_align2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_align2_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/r5_align2_tests.log | head; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for A in 8 32; do
  NT_ROW_ALIGN=$A timeout -k 10 300 python bench.py --workload qm9-32k --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/r5_align2.log 2>&1 || { tail -5 gpurun_out/r5_align2.log; exit 5; }
  echo "qm9-32k align $A: $(tail -1 gpurun_out/r5_align2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,1), "us/step", round(d["roofline"]["launch_us"],1), "us/launch")')"
done; done
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-embedded --no-training > gpurun_out/r5_align2.log 2>&1 || { tail -5 gpurun_out/r5_align2.log; exit 6; }
echo "default: $(tail -1 gpurun_out/r5_align2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["secondary"]["polymer-16"]; print(round(d["ms_per_step"]*1e3,1), "us/step", round(d["roofline"]["launch_us"],1), "us/launch | polymer", round(s["ms_per_step"]*1e3,1), "us/step", round(s["roofline"]["launch_us"],1))')"
