#!/bin/bash
# Novelty GPU pass: a pytest selection, then the config-3 novelty leg (default + 256M span) alone.
# Usage (through gpurun): [K="pytest -k expr"] bash tools/gpu_nov.sh TAG "TESTS" [VAR=value ...]
set -o pipefail
TAG=${1:-nov}; TESTS=${2:-tests/test_gpu_novelty.py}; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$TESTS" != "none" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS ${K:+-k "$K"} -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $OUT/pytest.log | head -20; echo "pytest failed rc=$rc"; exit $rc; }
fi
env "$@" timeout -k 10 300 python3 -u tools/nov_bench.py 4 > $OUT/nov.log 2>&1 || { tail -5 $OUT/nov.log; exit 1; }
tail -c 3000 $OUT/nov.log
