set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/bitcmp.py --save ship > gpurun_out/cl_bit.log 2>&1 || { tail -5 gpurun_out/cl_bit.log; exit 3; }
NT_LIB=variant:pre timeout -k 10 300 python tools/bitcmp.py --save pre >> gpurun_out/cl_bit.log 2>&1 || { tail -5 gpurun_out/cl_bit.log; exit 3; }
python tools/bitcmp.py --compare ship pre | tail -4
bash tools/gpu_check.sh
