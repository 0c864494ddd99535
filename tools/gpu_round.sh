#!/bin/bash
# One GPU pass for a round's evidence: the whole -m gpu suite, the default bench line (every leg), and
# a rocprofv3 kernel-trace summary of the headline step. Usage (via gpurun, repo root):
#   bash tools/gpu_round.sh TAG [tests|notests] [bench args...]
set -o pipefail
TAG=${1:-run}; shift
MODE=${1:-tests}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$MODE" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread --durations=15 > $OUT/pytest.log 2>&1
  rc=$?; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; exit $rc; }
fi
timeout -k 10 400 python -u bench.py "$@" > $OUT/bench.log 2>&1
rc=$?; tail -c 600 $OUT/bench.log; [ $rc -eq 0 ] || { echo "bench failed rc=$rc"; exit $rc; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --text 0 --novelty 0 --hub 0 --analytics 0 --append 0 --store 0 "$@" > $GRAFT_REPO_ROOT/$OUT/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
