#!/bin/bash
# parity of the raw minimize path, then timing A/B (tools/gpu_exp.sh) of the listed variants
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_raw.py tests/test_gpu_parity.py > gpurun_out/$TAG/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_exp.sh $TAG "$@"
