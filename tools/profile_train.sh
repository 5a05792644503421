#!/bin/bash
# Kernel-trace profile of the training step (tools/train_bench.py, kernel backward only).
# Usage (on the GPU box): tools/profile_train.sh [train_bench args...]
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof_train
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train -o run -- \
  python tools/train_bench.py --modes kernel --steps 10 "$@" > gpurun_out/prof_train/bench.log 2>&1
tail -3 gpurun_out/prof_train/bench.log
