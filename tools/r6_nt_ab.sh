#!/bin/bash
# A/B: nontemporal H[rev] gathers (ntq) / residual loads (ntr) in the fp32 layer kernel vs shipping
set -uo pipefail
mkdir -p gpurun_out
for W in polymer-16 qm9-32k qm9-4096; do for r in 1 2; do for L in "" variant:ntq variant:ntr; do
  NT_LIB=$L timeout -k 10 300 python bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/nt_ab.log 2>&1 || { tail -5 gpurun_out/nt_ab.log; exit 5; }
  echo "$W lib '$L': $(tail -1 gpurun_out/nt_ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["ms_per_step"]*1e3,1), "us/step", round(r["launch_us"],1), "us/launch")')"
done; done; done
