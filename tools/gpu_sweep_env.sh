#!/bin/bash
# Bench line per value of one environment knob (A/B of a tuning switch on the GPU box).
# Usage (repo root, through gpurun): bash tools/gpu_sweep_env.sh TAG VAR v1 v2 ... [-- bench args]
set -o pipefail
TAG=$1; VAR=$2; shift 2
VALS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VALS+=("$1"); shift; done
[ "$1" == "--" ] && shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for v in "${VALS[@]}"; do
  LOG=$OUT/${VAR}_${v//\//_}.log
  env $VAR=$v timeout -k 10 200 python -u bench.py --cpu-baseline 0 --raw-steps 0 "$@" > $LOG 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$VAR=$v rc=$rc"; tail -5 $LOG; exit $rc; }
  echo "$VAR=$v $(grep -o '"ms_per_step": [0-9.]*' $LOG | head -1)"
done
