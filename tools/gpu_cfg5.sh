#!/bin/bash
# Configs 1 and 2 (BASELINE.json configs[0], [1]) on one GPU: the bench line and a kernel trace of
# each. Usage (via gpurun): bash tools/gpu_cfg5.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
LEGS="--text 0 --novelty 0 --hub 0 --analytics 0 --append 0 --store 0 --cooccurrence 0 --setops 0 --canonicalize 0 --cpu-baseline 0"
for cfg in "config1 --progs-per-gpu 10000 --npcs 50000" "config2 --progs-per-gpu 100000 --npcs 500000"; do
  set -- $cfg; n=$1; shift
  timeout -k 10 300 python -u $R/bench.py $LEGS "$@" --steps 20 --warmup 3 > $OUT/$n.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/$n.log; exit $rc; }
  echo "$n $(grep '^{' $OUT/$n.log | tail -1 | cut -c1-260)"
  cd /tmp
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt_$n -o run -- python3 $R/bench.py $LEGS "$@" --steps 5 --warmup 2 --profile 0 > $OUT/kt_$n.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -3 $OUT/kt_$n.log; exit $rc; }
  cd $R
done
