#!/bin/bash
# profile packages for config 3 and config 5 at HEAD
set -uo pipefail
bash tools/profile_round.sh r6 zinc-4096-bf16 polymer-16 || exit 4
