#!/bin/bash
# config-4 raw step (pm_time, no per-kernel events) under environment variants, twice each, interleaved.
# Usage (via gpurun): bash tools/gpu_env5.sh TAG "VAR=v ..." ...
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for rep in 1 2; do
  for e in "X=0" "$@"; do
    r=$(env $e PM_PROF=0 timeout -k 10 120 python3 tools/pm_time.py 2>&1 | grep -o 'step_ms [0-9.]*') || exit 1
    echo "$rep [$e] $r" | tee -a $OUT/env.log
  done
done
