#!/bin/bash
# Round-end evidence on one GPU box: the -m gpu suite, smoke(), the default bench line, the training
# bench (tools/gpu_check.sh), then the per-workload rocprofv3 package (kernel stats + separate PMC
# passes, tools/profile_round.sh) and kernel stats of the fp32 and bf16 training steps.
# Usage: TAG=r3b bash tools/round_evidence.sh
set -uo pipefail
TAG=${TAG:-r3b}
TRAIN=1 bash tools/gpu_check.sh || exit $?
bash tools/profile_round.sh "$TAG" ${WORKLOADS:-qm9-4096 zinc-4096-bf16 polymer-16} || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_${TAG}_train -o run -- python3 tools/train_bench.py --modes kernel --steps 10 --warmup 3 > gpurun_out/prof_${TAG}_train.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_train.log; exit 7; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_${TAG}_train_bf16 -o run -- python3 tools/train_bench.py --kind zinc --h 512 --depth 5 --dtype bf16 --modes kernel --steps 10 --warmup 3 > gpurun_out/prof_${TAG}_train_bf16.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_train_bf16.log; exit 8; }
echo "evidence $TAG done"
