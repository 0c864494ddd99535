#!/bin/bash
# Serial phase timings of the raw minimize job (tools/pm_time.py, SYZGPU_PM_SERIAL=1: P before the sort)
# and a rocprofv3 kernel trace of the same run. Usage (through gpurun): bash tools/gpu_serial.sh TAG [VAR=value ...]
set -o pipefail
TAG=${1:-serial}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
env "$@" SYZGPU_PM_SERIAL=1 timeout -k 10 120 python3 tools/pm_time.py > $OUT/pm.log 2>&1 || { tail -5 $OUT/pm.log; exit 1; }
env "$@" timeout -k 10 120 python3 tools/pm_time.py >> $OUT/pm.log 2>&1 || { tail -5 $OUT/pm.log; exit 1; }
cat $OUT/pm.log
cd /tmp && env "$@" SYZGPU_PM_SERIAL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/pm_time.py > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
