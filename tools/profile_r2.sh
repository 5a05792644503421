#!/bin/bash
# Round-2 profile package: tools/profile_round.sh over the judged workloads, then the default bench
# line (driver command) for reference.  Usage: tools/profile_r2.sh <tag> [workload ...]
set -uo pipefail
TAG=${1:-r2}; shift || true
tools/profile_round.sh "$TAG" ${*:-qm9-4096 qm9-32k zinc-4096-bf16} || exit $?
