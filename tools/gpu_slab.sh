#!/bin/bash
# Slab-form P/M check: raw-minimize / novelty parity tests, then phase timings (pm_time.py): the slab
# form concurrent and serialized, its P timing modes (SYZGPU_RG_DBG 16: loads only, 32: + histogram and
# scan), and the region form for comparison.
# Usage (through gpurun): bash tools/gpu_slab.sh TAG ['pytest -k expr' | none]
set -o pipefail
TAG=${1:-slab}; K=${2:-raw or keyshard or minimize or config4 or novelty}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$K" != none ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1
  rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; exit $rc; }
fi
for v in "X=0" "SYZGPU_PM_SERIAL=1" "SYZGPU_PM_SERIAL=1 SYZGPU_RG_DBG=16" "SYZGPU_PM_SERIAL=1 SYZGPU_RG_DBG=32" "SYZGPU_PM_REGION=1" "SYZGPU_PM_REGION=1 SYZGPU_PM_SERIAL=1"; do
  echo "== $v" >> $OUT/pm.log
  env $v timeout -k 10 120 python3 tools/pm_time.py >> $OUT/pm.log 2>&1 || { tail -5 $OUT/pm.log; exit 1; }
done
grep -v amdgpu.ids $OUT/pm.log
