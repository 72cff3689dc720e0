set -o pipefail
for cfg in "X=0" "PBF_NTT_PASSES=7,7,6" "PBF_NTT_PASSES=6,7,7" "PBF_NTT_PASSES=8,6,6" "PBF_NTT_PASSES=7,7,6 PBF_NTT_TILE=8192" "PBF_NTT_PASSES=9,11" "X=0"; do
  out=$(env $cfg timeout -k 10 120 python bench.py --log-n 20 --batch 32 --steps 20 --warmup 3 --no-cpu --no-extra --no-traffic 2>/dev/null) || { echo "$cfg failed"; continue; }
  echo "$out" | python -c "import json,sys; d=json.load(sys.stdin); print('%-44s 2^20 x 32: %.4f ms'%('$cfg',d['ms_per_step']))"
done
