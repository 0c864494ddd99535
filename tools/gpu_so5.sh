#!/bin/bash
# set-op parity, then the set-op leg with the look-back merge (default) and round 4's gapped image + compaction
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "setop or store or minimize_golden" > $OUT/t.log 2>&1
rc=$?; tail -1 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $OUT/t.log | head; exit $rc; }
for e in "X=0" "SYZGPU_SO_GAP=1"; do
  env $e timeout -k 10 300 python -u tools/leg_time.py setops --steps 6 --cpu-baseline 0 > $OUT/so_$e.log 2>&1 || { tail -3 $OUT/so_$e.log; exit 1; }
  python3 - $OUT/so_$e.log "$e" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], {k: (v["ms_per_batch"], v["kernels_ms"], v["roofline"]["frac"]) for k, v in d["ops"].items()})
PY
done
