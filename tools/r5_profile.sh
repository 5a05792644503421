#!/bin/bash
# Round-5 profile package: per-workload rocprofv3 trace/stats + separate PMC passes + bench line, and
# the training step's kernel trace
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
bash tools/profile_round.sh r5 qm9-4096 zinc-4096-bf16 polymer-16 || exit 3
bash tools/profile_train.sh || exit 4
