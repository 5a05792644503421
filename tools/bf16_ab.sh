#!/bin/bash
# config-3 bf16 update launch time, fused (tile plan + aggregation) vs unfused (NT_FUSED=0)
set -uo pipefail
J='import json,sys; d=json.loads(sys.stdin.readlines()[-1]); r=d["roofline"]; print("%.3e" % d["value"], "%.3f ms" % d["ms_per_step"], "launch %.1f us" % (r["launch_ms"]*1e3))'
for v in NT_FUSED=1 NT_FUSED=0 NT_FUSED=1; do
  env $v timeout -k 10 200 python bench.py --workload zinc-4096-bf16 --steps 20 --warmup 5 --no-cpu-baseline --no-embedded > gpurun_out/bf16_ab.log 2>&1 || exit 3
  echo -n "$v: "; python -c "$J" < gpurun_out/bf16_ab.log
done
