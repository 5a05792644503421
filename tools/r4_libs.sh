set -uo pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in ${LIBS:-base}; do
  if [ $v = base ]; then L=""; else L=variant:$v; fi
  NT_LIB=$L timeout -k 10 300 python bench.py --workload qm9-4096 --steps 50 --warmup 10 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/bl_$v.log 2>&1 || { tail -5 gpurun_out/bl_$v.log; exit 4; }
  echo "$v: $(tail -1 gpurun_out/bl_$v.log | grep -o '"ms_per_step": [0-9.]*\|"launch_us": [0-9.]*' | tr '\n' ' ')"
  NT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pl_$v -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/pl_$v.log 2>&1 || { tail -5 gpurun_out/pl_$v.log; exit 7; }
  python tools/trace_gaps.py $(find gpurun_out/pl_$v -name "*kernel_trace.csv" | head -1) --last 120 | head -6
done
