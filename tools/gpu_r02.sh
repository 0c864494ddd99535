#!/bin/bash
# Round-2 GPU pass: raw-pipeline parity tests, the bench line, and a rocprofv3 kernel-trace summary of
# the same bench command. Usage (through gpurun, from the repo root): bash tools/gpu_r02.sh TAG [tests] [bench args...]
set -o pipefail
TAG=${1:-run}; shift
TESTS=${1:-tests/test_gpu_raw.py}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$TESTS" != "none" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; exit $rc; }
fi
timeout -k 10 300 python -u bench.py "$@" > $OUT/bench.log 2>&1
rc=$?; tail -c 1200 $OUT/bench.log; [ $rc -eq 0 ] || { echo "bench failed rc=$rc"; exit $rc; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --text 0 --novelty 0 --hub 0 --analytics 0 --append 0 --store 0 "$@" > $GRAFT_REPO_ROOT/$OUT/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; f=$(find $GRAFT_REPO_ROOT/$OUT/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -25 "$f" | cut -d, -f1-8; exit $rc
