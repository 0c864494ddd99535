#!/bin/bash
# the whole GPU test suite (as the driver runs it at round end), log under gpurun_out/TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; exit $rc
