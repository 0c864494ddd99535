#!/bin/bash
# Headline step under alternating env settings, twice each (noise check). Usage: bash tools/gpu_step_env_ab.sh TAG "SET_A" "SET_B"
set -o pipefail
TAG=${1:-envab}; A=$2; B=$3
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for SET in "$A" "$B" "$A" "$B"; do
  i=$((i+1))
  env $SET timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --novelty 0 --text 0 --hub 0 --analytics 0 \
      --append 0 --store 0 --cpu-baseline 0 > $OUT/b$i.log 2>&1 || { tail -5 $OUT/b$i.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$OUT/b$i.log') if l.startswith('{')][-1])
print('[$SET]', d['ms_per_step'], d['kernels_ms_per_step_serialized_pass'].get('pmin'), d['kernels_ms_per_step_serialized_pass'].get('pmin_small'))" | tee -a $OUT/ab.log
done
