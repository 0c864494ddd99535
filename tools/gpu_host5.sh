#!/bin/bash
# The raw minimize step (no per-kernel events) with and without speculation, a kernel trace of it,
# and the parity of the raw path. Usage (via gpurun): bash tools/gpu_host5.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_raw.py > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for e in "PM_PROF=0" "PM_PROF=0 SYZGPU_PM_SPEC=0"; do
  echo "== $e" >> $OUT/pm.log
  env $e timeout -k 10 120 python3 tools/pm_time.py >> $OUT/pm.log 2>&1 || exit 1
done
cut -c1-200 $OUT/pm.log
cd /tmp
PM_PROF=0 PM_K=2 PM_W=2 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 $R/tools/pm_time.py > $OUT/kt.log 2>&1
rc=$?; tail -1 $OUT/kt.log; exit $rc
