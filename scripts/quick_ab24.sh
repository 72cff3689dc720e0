#!/bin/bash
# A/B timing of env-var variants of the 2^24 x 2 bench only: quick_ab24.sh "ENV=.. ENV2=.." ...
set -o pipefail
for cfg in "$@"; do
  out=$(env $cfg timeout -k 10 120 python bench.py --log-n 24 --batch 2 --steps 20 --warmup 3 --no-cpu --no-extra) || exit 1
  echo "$out" | python -c "import json,sys; d=json.load(sys.stdin); print('%-50s 2^24 x 2: %.4f ms  %.1f GB/s  frac %.4f'%('$cfg',d['ms_per_step'],d['roofline']['achieved'],d['roofline']['frac']))"
done
