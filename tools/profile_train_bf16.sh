set -uo pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_train_bf16 -o run -- python3 tools/train_bench.py --kind zinc --h 512 --depth 5 --dtype bf16 --modes kernel --steps 10 --warmup 3 > gpurun_out/prof_train_bf16.log 2>&1 || { tail -20 gpurun_out/prof_train_bf16.log; exit 7; }
F=$(find gpurun_out/prof_train_bf16 -name "*kernel_stats.csv" | head -1); head -16 "$F" | cut -d, -f1-4
