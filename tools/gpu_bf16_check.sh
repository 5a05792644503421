set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16_backward.py tests/test_gpu_bf16.py -x -v --timeout 120 --timeout-method thread > gpurun_out/bf_tests.log 2>&1
rc=$?; tail -3 gpurun_out/bf_tests.log; grep -E "FAILED|ERROR|Error" gpurun_out/bf_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
for W in kernel library; do
  NT_WGRAD=$W timeout -k 10 300 python tools/train_bench.py --kind zinc --h 512 --depth 5 --dtype bf16 --modes kernel > gpurun_out/train_bf16_$W.log 2>&1 || { tail -20 gpurun_out/train_bf16_$W.log; exit 6; }
  echo "NT_WGRAD=$W"; tail -2 gpurun_out/train_bf16_$W.log
done
