#!/bin/bash
# One short GPU call: the raw-minimize parity tests, pm_time (serialized and concurrent) and a kernel
# trace of the concurrent step for tools/timeline.py.
# Usage (through gpurun): bash tools/gpu_quick2.sh TAG
set -o pipefail
TAG=${1:-quick2}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_raw.py tests/test_gpu_configs.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for e in "SYZGPU_PM_SERIAL=1" "X=0"; do
  echo "== $e" >> $OUT/pm.log
  env $e timeout -k 10 120 python3 $R/tools/pm_time.py 2>&1 | grep -v amdgpu.ids >> $OUT/pm.log || exit 1
done
cut -c1-400 $OUT/pm.log
cd /tmp
PM_K=2 PM_W=2 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 $R/tools/pm_time.py > $OUT/kt.log 2>&1
rc=$?; [ $rc -eq 0 ] || tail -3 $OUT/kt.log; exit $rc
