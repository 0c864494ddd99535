#!/bin/bash
# Headline-step A/B: bench.py's step only (no side legs, no CPU baseline) under each "VAR=value ..." setting
# given (the first run has none). Usage (repo root, via gpurun): bash tools/gpu_step_ab.sh TAG "SET1" "SET2" ...
set -o pipefail
TAG=${1:-stepab}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for SET in "" "$@"; do
  i=$((i+1))
  echo "== [$SET]" | tee -a $OUT/ab.log
  env $SET timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 3 --novelty 0 --text 0 --hub 0 --analytics 0 \
      --append 0 --store 0 --cpu-baseline 0 > $OUT/b$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "run $i rc=$rc"; tail -5 $OUT/b$i.log; exit $rc; }
  python3 -c "
import json
d=json.loads([l for l in open('$OUT/b$i.log') if l.startswith('{')][-1])
print(d['ms_per_step'], {k: v for k, v in d['kernels_ms_per_step_serialized_pass'].items()})" | tee -a $OUT/ab.log
done
