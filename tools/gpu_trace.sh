#!/bin/bash
# One GPU call: the store/gate tests, the NewInput timings (tools/append_time.py) and a kernel trace of the
# raw minimize job (pm_time.py, concurrent) for the step's timeline (tools/timeline.py reads it).
# Usage (through gpurun): bash tools/gpu_trace.sh TAG
set -o pipefail
TAG=${1:-trace}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_append.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/append_time.py > $OUT/append.log 2>&1
rc=$?; tail -c 2500 $OUT/append.log; [ $rc -eq 0 ] || exit $rc
cd /tmp
PM_K=2 PM_W=2 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 $R/tools/pm_time.py > $OUT/kt.log 2>&1
rc=$?; tail -3 $OUT/kt.log; [ $rc -eq 0 ] || exit $rc
for e in "X=0" "SYZGPU_GS_HIPRI=1"; do
  echo "== $e" >> $OUT/pm.log
  env $e timeout -k 10 120 python3 $R/tools/pm_time.py >> $OUT/pm.log 2>&1 || exit 1
done
cat $OUT/pm.log | cut -c1-400
SYZGPU_GS_HIPRI=1 PM_K=2 PM_W=2 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/kth -o run -- python3 $R/tools/pm_time.py > $OUT/kth.log 2>&1
rc=$?; tail -3 $OUT/kth.log; exit $rc
