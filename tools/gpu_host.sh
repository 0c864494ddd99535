#!/bin/bash
# One short GPU call: host-side planning times (SYZGPU_HOST_TIMING) and pm_time concurrent + a trace.
set -o pipefail
TAG=${1:-host}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
SYZGPU_HOST_TIMING=1 PM_K=3 PM_W=2 timeout -k 10 120 python3 $R/tools/pm_time.py > $OUT/host.log 2>&1 || exit 1
grep "\[host\]" $OUT/host.log | tail -16
for e in "SYZGPU_PM_SERIAL=1" "X=0"; do
  echo "== $e" >> $OUT/pm.log
  env $e timeout -k 10 120 python3 $R/tools/pm_time.py 2>&1 | grep -v amdgpu.ids >> $OUT/pm.log || exit 1
done
cut -c1-400 $OUT/pm.log
cd /tmp
PM_K=2 PM_W=2 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 $R/tools/pm_time.py > $OUT/kt.log 2>&1
rc=$?; [ $rc -eq 0 ] || tail -3 $OUT/kt.log; exit $rc
