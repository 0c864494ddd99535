#!/bin/bash
# One GPU call for a checkpoint: the full -m gpu suite, the NewInput timings with the phase split
# (tools/append_time.py, SYZGPU_PHASE_TIMING=1), a kernel trace of the raw minimize job and a bench line.
# Usage (through gpurun): bash tools/gpu_check2.sh TAG
set -o pipefail
TAG=${1:-check2}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; exit $rc; }
SYZGPU_PHASE_TIMING=1 timeout -k 10 200 python3 tools/append_time.py > $OUT/append.log 2>&1
rc=$?; grep -v "^\[phase\]" $OUT/append.log | tail -c 2000; [ $rc -eq 0 ] || exit $rc
cd /tmp
PM_K=2 PM_W=2 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 $R/tools/pm_time.py > $OUT/kt.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/kt.log; exit $rc; }
cd $R
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 > $OUT/bench.log 2>&1
rc=$?; tail -c 1500 $OUT/bench.log; exit $rc
