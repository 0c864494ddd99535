#!/bin/bash
# parity of the default library (raw minimize, set ops, novelty), then timing A/B of library variants
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_raw.py tests/test_gpu_parity.py tests/test_gpu_novelty.py > gpurun_out/$TAG/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/tests.log; [ $rc -eq 0 ] || exit $rc
for E in "$@"; do
  L=${E%%|*}
  [ "$L" = base ] && continue
  env SYZGPU_LIB=$GRAFT_REPO_ROOT/syzkaller_amd/libsyzgpu_$L.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_raw.py > gpurun_out/$TAG/tests_$L.log 2>&1
  rc=$?; echo "$L: $(tail -1 gpurun_out/$TAG/tests_$L.log)"; [ $rc -eq 0 ] || exit $rc
done
bash tools/gpu_exp.sh $TAG "$@" || exit $?
timeout -k 10 300 python -u tools/leg_time.py canonicalize --steps 6 --cpu-baseline 0 > gpurun_out/$TAG/canon.log 2>&1; tail -c 1200 gpurun_out/$TAG/canon.log
