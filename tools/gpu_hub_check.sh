set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_hubs.py tests/test_gpu_parity.py tests/test_gpu_backward.py tests/test_gpu_fused.py -k "hub or polymer" -x -v --timeout 120 --timeout-method thread > gpurun_out/hub_tests.log 2>&1
rc=$?; tail -5 gpurun_out/hub_tests.log; grep -E "FAILED|ERROR|Error" gpurun_out/hub_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload polymer-16 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-embedded --no-training > gpurun_out/bench_poly.log 2>&1 || { tail -20 gpurun_out/bench_poly.log; exit 4; }
tail -1 gpurun_out/bench_poly.log | cut -c1-1200
