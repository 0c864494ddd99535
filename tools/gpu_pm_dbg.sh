#!/bin/bash
# Serial per-kernel times of the raw minimize job (tools/pm_time.py) under SYZGPU_PM_DBG settings
# (1: no table updates, 2: no winner emit, 3: both, 4: no hash windows, 64: hash walked not probed).
# Usage (repo root, through gpurun): bash tools/gpu_pm_dbg.sh TAG "DBG1 DBG2 ..." [VAR=value ...]
set -o pipefail
TAG=${1:-pmdbg}; DBGS=${2:-"0 1 3"}; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp SYZGPU_PM_SERIAL=1
for D in $DBGS; do
  env "$@" SYZGPU_PM_DBG=$D timeout -k 10 120 python3 tools/pm_time.py >> $OUT/pm.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "dbg $D rc=$rc"; tail -5 $OUT/pm.log; exit $rc; }
done
grep step_ms $OUT/pm.log
