set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for r in 1 2; do for v in ${LIBS:-base nt2}; do
  if [ $v = base ]; then L=""; else L=variant:$v; fi
  NT_LIB=$L timeout -k 10 300 python bench.py --workload ${WLB:-qm9-4096} --steps 100 --warmup 10 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/b2_$v.log 2>&1 || exit 4
  echo "$v r$r: $(tail -1 gpurun_out/b2_$v.log | grep -o '"ms_per_step": [0-9.]*\|"launch_us": [0-9.]*' | tr '\n' ' ')"
done; done
