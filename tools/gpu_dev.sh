#!/bin/bash
# Development GPU pass: a pytest selection, then serial + concurrent phase timings of the raw minimize
# job (tools/pm_time.py). Usage (through gpurun): bash tools/gpu_dev.sh TAG "TESTS" [VAR=value ...]
set -o pipefail
TAG=${1:-dev}; TESTS=${2:-tests/test_gpu_raw.py}; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$TESTS" != "none" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; exit $rc; }
fi
env "$@" SYZGPU_PM_SERIAL=1 timeout -k 10 120 python3 tools/pm_time.py > $OUT/pm.log 2>&1 || { tail -5 $OUT/pm.log; exit 1; }
env "$@" timeout -k 10 120 python3 tools/pm_time.py >> $OUT/pm.log 2>&1 || { tail -5 $OUT/pm.log; exit 1; }
grep step_ms $OUT/pm.log
