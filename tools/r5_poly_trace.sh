#!/bin/bash
# per-dispatch kernel trace of the polymer-16 forward (which chunked reduce costs what)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/poly_trace; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/t -o run -- python3 bench.py --workload polymer-16 --steps 3 --warmup 2 --no-cpu-baseline --no-secondary --no-embedded --no-training > $OUT/log 2>&1 || { tail -5 $OUT/log; exit 3; }
F=$(find $OUT/t -name "*kernel_trace.csv" | head -1)
python3 - "$F" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows[-40:]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f'{r["Kernel_Name"][:60]:60s} grid {r.get("Grid_Size_X", r.get("Grid_Size", "?")):>9s} {d:9.1f} us')
PY
tail -1 $OUT/log | cut -c1-300
