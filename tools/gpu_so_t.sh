#!/bin/bash
# set-op parity tests, then the set-op leg's timing (dev tooling). Usage (via gpurun): bash tools/gpu_so_t.sh TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread $(grep -ln "setop" tests/test_gpu_*.py) > $OUT/t.log 2>&1
rc=$?; tail -1 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $OUT/t.log | head; exit $rc; }
timeout -k 10 300 python -u tools/leg_time.py setops --steps 6 --cpu-baseline 0 > $OUT/so.log 2>&1 || { tail -3 $OUT/so.log; exit 1; }
python3 - $OUT/so.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print({k: (v["ms_per_batch"], v["kernels_ms"], v["roofline"]["frac"]) for k, v in d["ops"].items()})
PY
