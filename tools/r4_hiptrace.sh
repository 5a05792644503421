set -uo pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/ph -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/ph.log 2>&1 || { tail -5 gpurun_out/ph.log; exit 7; }
ls gpurun_out/ph
