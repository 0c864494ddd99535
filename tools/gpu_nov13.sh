#!/bin/bash
# novelty A/B: parity with 13-bit direct windows, then the config-3 leg with the default and with 13 bits
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
SYZGPU_NW_BITS=13 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_novelty.py > $OUT/t13.log 2>&1
rc=$?; tail -1 $OUT/t13.log; [ $rc -eq 0 ] || exit $rc
for e in "X=0" "SYZGPU_NW_BITS=13"; do
  env $e timeout -k 10 300 python -u tools/leg_time.py novelty --steps 6 --cpu-baseline 0 --novelty-wide 1 > $OUT/nov_$e.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/nov_$e.log; exit $rc; }
  python3 - $OUT/nov_$e.log "$e" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], json.dumps(d)[:1500])
PY
done
