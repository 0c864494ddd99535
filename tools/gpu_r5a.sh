#!/bin/bash
# Round-5 check: parity of the default library (raw minimize incl. the speculative plan, set ops,
# novelty, two ranks), the step with and without the speculative P, configs 1/2, a kernel trace of
# the step, the novelty 13-bit A/B and the canonicalize leg. Usage (via gpurun): bash tools/gpu_r5a.sh TAG
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_raw.py tests/test_gpu_parity.py tests/test_gpu_multirank.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_exp.sh $TAG base "base|SYZGPU_PM_SPEC=0" || exit $?
LEGS="--text 0 --novelty 0 --hub 0 --analytics 0 --append 0 --store 0 --cooccurrence 0 --setops 0 --canonicalize 0 --cpu-baseline 0"
for cfg in "config1 --progs-per-gpu 10000 --npcs 50000" "config2 --progs-per-gpu 100000 --npcs 500000"; do
  set -- $cfg; n=$1; shift
  timeout -k 10 300 python -u bench.py $LEGS "$@" --steps 20 --warmup 3 > $OUT/$n.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/$n.log; exit $rc; }
  echo "$n $(grep '^{' $OUT/$n.log | tail -1 | cut -c1-200)"
done
cd /tmp
PM_K=2 PM_W=2 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 $R/tools/pm_time.py > $OUT/kt.log 2>&1
rc=$?; tail -2 $OUT/kt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt1 -o run -- python3 $R/bench.py $LEGS --progs-per-gpu 10000 --npcs 50000 --steps 5 --warmup 2 --profile 0 > $OUT/kt1.log 2>&1
rc=$?; tail -2 $OUT/kt1.log; [ $rc -eq 0 ] || exit $rc
cd $R
bash tools/gpu_nov13.sh $TAG || exit $?
timeout -k 10 300 python -u tools/leg_time.py canonicalize --steps 6 --cpu-baseline 0 > $OUT/canon.log 2>&1; rc=$?; tail -c 1500 $OUT/canon.log; exit $rc
