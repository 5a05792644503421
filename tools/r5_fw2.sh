#!/bin/bash
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 python -u tools/fw_check.py --mols 32768 --rev nodes --rounds 3 > gpurun_out/fw2_q32k.log 2>&1; grep -E "bit-exact|median|V=" gpurun_out/fw2_q32k.log
timeout -k 10 240 python -u tools/fw_check.py --kind zinc --mols 4096 --h 512 --dtype bf16 --rounds 3 > gpurun_out/fw2_zinc.log 2>&1; grep -E "bit-exact|median|V=|Error" gpurun_out/fw2_zinc.log; tail -3 gpurun_out/fw2_zinc.log
