#!/bin/bash
# A/B timing of env-var variants of the 2^20 x 32 and 2^24 x 2 bench: quick_ab.sh "ENV=.. ENV2=.." "ENV=.." ...
set -o pipefail
for cfg in "$@"; do
  for L in "20 32" "24 2"; do
    set -- $L
    out=$(env $cfg timeout -k 10 120 python bench.py --log-n $1 --batch $2 --steps 20 --warmup 3 --no-cpu --no-extra --no-traffic) || exit 1
    echo "$out" | python -c "import json,sys; d=json.load(sys.stdin); print('%-40s 2^%s x %s: %.4f ms  %.1f GB/s  frac %.4f'%('$cfg',$1,$2,d['ms_per_step'],d['roofline']['achieved'],d['roofline']['frac']))"
  done
done
