#!/bin/bash
# A/B timing of env-var variants of the 2^24 x 2 NTT step: quick_ab24.sh "ENV=.." ...
set -o pipefail
for cfg in "$@"; do
  out=$(env $cfg timeout -k 10 120 python bench.py --log-n 24 --batch 2 --steps 20 --warmup 3 --no-cpu --no-extra --no-traffic 2>/dev/null) || exit 1
  echo "$out" | python -c "import json,sys; d=json.load(sys.stdin); print('%-48s 2^24 x 2: %.4f ms  frac %.4f'%('$cfg',d['ms_per_step'],d['roofline']['frac']))"
done
