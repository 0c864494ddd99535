#!/bin/bash
# Timing experiments on the raw minimize job (dev tooling): per entry "LIBTAG[|VAR=v ...]" the serial
# per-kernel times and the concurrent step of tools/pm_time.py (no parity: variants may be timing-only).
# Usage (repo root, via gpurun): bash tools/gpu_exp.sh TAG ENTRY...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for E in "$@"; do
  i=$((i+1))
  LT=${E%%|*}; ENVS=""; [ "$E" != "$LT" ] && ENVS=${E#*|}
  LIB=$GRAFT_REPO_ROOT/syzkaller_amd/libsyzgpu.so; [ "$LT" != "base" ] && LIB=$GRAFT_REPO_ROOT/syzkaller_amd/libsyzgpu_$LT.so
  for ser in 1 0; do
    echo "== $i [$E] serial=$ser" >> $OUT/pm.log
    env SYZGPU_LIB=$LIB $ENVS SYZGPU_PM_SERIAL=$ser timeout -k 10 150 python3 tools/pm_time.py > $OUT/pm${i}_${ser}.log 2>&1
    rc=$?; grep step_ms $OUT/pm${i}_${ser}.log | cut -c1-600 >> $OUT/pm.log; [ $rc -eq 0 ] || { tail -5 $OUT/pm${i}_${ser}.log; exit $rc; }
  done
done
cat $OUT/pm.log
