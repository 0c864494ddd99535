#!/bin/bash
# The whole GPU test suite in one process, log under gpurun_out/TAG. Usage: bash tools/gpu_full_tests.sh TAG
set -o pipefail
TAG=${1:-full}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; grep -E "FAILED|ERROR" $OUT/pytest.log | head -20; exit $rc
