#!/bin/bash
# wide-window C / D sums after the quad select fix: single lanes (default) vs quads vs SEQ 32
set -o pipefail
for i in 1 2; do
  for V in default quad seq32; do
    unset PBF_MSM_CD_QUAD PBF_MSM_CD_SEQ32
    [ $V = quad ] && export PBF_MSM_CD_QUAD=1
    [ $V = seq32 ] && export PBF_MSM_CD_SEQ32=1
    echo "$V $(timeout -k 10 200 python scripts/probe_msm_fixed.py 24 5 | tail -1)"
  done
done
