#!/bin/bash
# kernel-trace --stats of one workload's bench run (round-4 iteration helper).  Usage: WL=polymer-16 [NT_LIB=..] bash tools/r4_prof_wl.sh
set -uo pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
W=${WL:-polymer-16}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/pw_$W -o run -- python3 bench.py --workload $W --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/pw_$W.log 2>&1 || { tail -5 gpurun_out/pw_$W.log; exit 7; }
F=$(find gpurun_out/pw_$W -name "*kernel_stats.csv" | head -1); head -14 "$F" | cut -d, -f1-4
