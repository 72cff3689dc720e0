#!/bin/bash
# Round 6: rehearsal of the driver's N > 1 bench path on the final tree, on a
# one-GPU box: N ranks share the GPU, collectives over gloo with host staging (timings meaningless
# by construction; the point is that every rank completes the sharded NTT steps and the sharded
# prove, holds the same proof, and the line carries config.world / config.backend).
set -o pipefail
mkdir -p gpurun_out/r06
for cfg in "2 16,20,24" "4 16,20"; do
  set -- $cfg
  N=$1
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29600 + N)) bench.py --gpus $N --backend gloo --steps 3 --warmup 1 --no-cpu --no-traffic \
    --prove-log-n $2 > gpurun_out/r06/gloo_n$N.json 2> gpurun_out/r06/gloo_n$N.err || exit $?
  python -c "
import json
d = json.loads([l for l in open('gpurun_out/r06/gloo_n$N.json') if l.startswith('{')][-1])
print('N=$N', 'world', d['config'].get('world'), 'backend', d['config'].get('backend'), 'ms/step', round(d['ms_per_step'], 2),
      {k: (v.get('ranks_agree'), v.get('error')) for k, v in d.get('extra', {}).get('config5_prove_sharded', {}).items()})
"
done
