#!/bin/bash
# Rehearsal of the driver's N > 1 bench path on a one-GPU box: N ranks share the GPU, collectives
# over gloo with host staging (timings meaningless by construction; the point is that every rank
# completes the sharded NTT steps and the sharded prove and holds the same proof).
set -o pipefail
mkdir -p gpurun_out/r04g2
for N in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29500 + N)) bench.py --gpus $N --backend gloo --steps 3 --warmup 1 --no-cpu --no-traffic \
    --prove-log-n 16,20 > gpurun_out/r04g2/gloo_n$N.json 2> gpurun_out/r04g2/gloo_n$N.err || exit $?
done
