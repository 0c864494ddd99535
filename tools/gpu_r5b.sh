#!/bin/bash
# Parity (raw minimize, set ops / canonicalize, novelty, two ranks), the step's timing and kernel
# trace, and the canonicalize leg. Usage (via gpurun): bash tools/gpu_r5b.sh TAG [gpu_exp entries...]
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_raw.py tests/test_gpu_parity.py tests/test_gpu_novelty.py tests/test_gpu_multirank.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_exp.sh $TAG base "$@" || exit $?
cd /tmp
PM_K=2 PM_W=2 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 $R/tools/pm_time.py > $OUT/kt.log 2>&1
rc=$?; tail -1 $OUT/kt.log; [ $rc -eq 0 ] || exit $rc
cd $R
timeout -k 10 300 python -u tools/leg_time.py canonicalize --steps 6 --cpu-baseline 0 > $OUT/canon.log 2>&1; rc=$?; tail -c 1500 $OUT/canon.log; exit $rc
