#!/bin/bash
# Configs 1 / 2 bench lines and the config-4 raw step (pm_time, no events) per library variant.
# Usage (via gpurun): bash tools/gpu_cfgab.sh TAG ENTRY...   (ENTRY: LIBTAG[|VAR=v ...], "base": the default library)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
LEGS="--text 0 --novelty 0 --hub 0 --analytics 0 --append 0 --store 0 --cooccurrence 0 --setops 0 --canonicalize 0 --cpu-baseline 0"
i=0
for E in "$@"; do
  i=$((i+1)); LT=${E%%|*}; ENVS="X=0"; [ "$E" != "$LT" ] && ENVS=${E#*|}
  LIB=$R/syzkaller_amd/libsyzgpu.so; [ "$LT" != base ] && LIB=$R/syzkaller_amd/libsyzgpu_$LT.so
  for cfg in "config1 --progs-per-gpu 10000 --npcs 50000" "config2 --progs-per-gpu 100000 --npcs 500000"; do
    set -- $cfg; n=$1; shift
    env SYZGPU_LIB=$LIB $ENVS timeout -k 10 300 python -u $R/bench.py $LEGS "$@" --steps 20 --warmup 3 > $OUT/${i}_$n.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/${i}_$n.log; exit $rc; }
    echo "$E $n $(grep '^{' $OUT/${i}_$n.log | tail -1 | grep -o '"ms_per_step": [0-9.]*')"
  done
  env SYZGPU_LIB=$LIB $ENVS PM_PROF=0 timeout -k 10 120 python3 $R/tools/pm_time.py > $OUT/${i}_pm.log 2>&1 || exit 1
  echo "$E config4 $(grep -o 'step_ms [0-9.]*' $OUT/${i}_pm.log)"
done
