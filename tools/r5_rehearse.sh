#!/bin/bash
# rehearsal of bench.py's N>1 path on one GPU: two ranks on cuda:0 (gloo bookkeeping), the driver's
# launcher and flags; not a scaling measurement
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 20 --warmup 5 --same-device --dist-backend gloo > gpurun_out/r5_rehearse.log 2>&1 || { tail -20 gpurun_out/r5_rehearse.log; exit 3; }
grep '^{"metric"' gpurun_out/r5_rehearse.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["n_gpus"], d["value"], d["ms_per_step"], d["prewarm_s"], d["roofline"]["launches_timed"], d["config"]["parallelism"])'
