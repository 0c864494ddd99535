#!/bin/bash
# One GPU call for a round checkpoint with evidence: the full -m gpu suite, the NewInput timings with the
# phase split (tools/append_time.py), then tools/gpu_final.sh (the default bench line with every leg,
# rocprofv3 --kernel-trace --stats of the headline step, FETCH_SIZE / WRITE_SIZE passes).
# Usage (through gpurun): bash tools/gpu_check3.sh TAG
set -o pipefail
TAG=${1:-check3}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; exit $rc; }
SYZGPU_PHASE_TIMING=1 timeout -k 10 200 python3 tools/append_time.py > $OUT/append.log 2>&1
rc=$?; grep -v "^\[phase\]" $OUT/append.log | tail -c 1500; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_final.sh $TAG/final
