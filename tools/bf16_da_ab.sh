set -uo pipefail
mkdir -p gpurun_out
for R in 1 2; do
for DA in kernel library; do
  NT_BF16_DA=$DA timeout -k 10 300 python tools/train_bench.py --kind zinc --h 512 --depth 5 --dtype bf16 --modes kernel --warmup-s 1 --steps 30 > gpurun_out/bfda_$DA.log 2>&1 || { tail -20 gpurun_out/bfda_$DA.log; exit 6; }
  echo "NT_BF16_DA=$DA round $R: $(tail -1 gpurun_out/bfda_$DA.log)"
done
done
