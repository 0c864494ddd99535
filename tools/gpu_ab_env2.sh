#!/bin/bash
# pm_time (concurrent) under env variants, interleaved twice (dev tooling). Usage: bash tools/gpu_ab_env2.sh TAG "A=1" "B=2" ...
set -o pipefail
TAG=${1:-ab}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for rep in 1 2; do
  for e in "$@"; do
    echo "== $e ($rep)" >> $OUT/pm.log
    env $e timeout -k 10 120 python3 tools/pm_time.py 2>&1 | grep -v amdgpu.ids >> $OUT/pm.log || exit 1
  done
done
cut -c1-200 $OUT/pm.log
