#!/bin/bash
# One GPU-box pass: parity tests, bench line, rocprofv3 kernel-trace summary of the same bench command.
# Usage (from the repo root, through gpurun): bash tools/gpu_check.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; exit $rc; }
timeout -k 10 300 python -u bench.py "$@" > $OUT/bench.log 2>&1
rc=$?; tail -c 3000 $OUT/bench.log; [ $rc -eq 0 ] || { echo "bench failed rc=$rc"; exit $rc; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --raw-steps 0 "$@" > $GRAFT_REPO_ROOT/$OUT/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
