#!/bin/bash
# A/B of pk kernel variants on the default bench (config 2).  Usage: tools/pk_ab.sh "ENV=a" "ENV=b" ...
set -uo pipefail
J='import json,sys; d=json.loads(sys.stdin.readlines()[-1]); r=d["roofline"]; print("%.3e" % d["value"], "%.3f ms" % d["ms_per_step"], "launch %.1f us" % r["launch_us"])'
i=0
for v in "$@"; do
  env $v timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-embedded --no-secondary > gpurun_out/pk_ab_$i.log 2>&1 || exit 3
  echo -n "$v: "; python -c "$J" < gpurun_out/pk_ab_$i.log
  i=$((i+1))
done
