#!/bin/bash
# set-op variants: parity (tests/test_gpu_parity.py set-op cases) and the setops_triage leg per library
# Usage (repo root, via gpurun): bash tools/gpu_so.sh TAG LIB...   (LIB base = the default library)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for L in "$@"; do
  LIB=$GRAFT_REPO_ROOT/syzkaller_amd/libsyzgpu.so; [ "$L" != base ] && LIB=$GRAFT_REPO_ROOT/syzkaller_amd/libsyzgpu_$L.so
  env SYZGPU_LIB=$LIB timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "setop or canonicalize" > $OUT/t_$L.log 2>&1
  rc=$?; echo "$L tests: $(tail -1 $OUT/t_$L.log)" | tee -a $OUT/so.log; [ $rc -eq 0 ] || exit $rc
  env SYZGPU_LIB=$LIB timeout -k 10 300 python -u tools/leg_time.py setops --steps 6 --cpu-baseline 0 > $OUT/l_$L.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/l_$L.log; exit $rc; }
  python3 - $OUT/l_$L.log $L <<'PY' | tee -a $OUT/so.log
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], {k: (v["ms_per_batch"], v["kernels_ms"], v["roofline"]["frac"]) for k, v in d["ops"].items()})
PY
done
timeout -k 10 300 python -u tools/leg_time.py canonicalize --steps 6 --cpu-baseline 0 > $OUT/canon.log 2>&1
rc=$?; tail -c 1500 $OUT/canon.log; exit $rc
