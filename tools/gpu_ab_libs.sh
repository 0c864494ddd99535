#!/bin/bash
# A/B of library variants and env settings on the raw minimize job: per entry "LIBTAG[|VAR=v VAR2=v]"
# (LIBTAG "base" = syzkaller_amd/libsyzgpu.so, else libsyzgpu_LIBTAG.so): the raw-pipeline parity
# tests, the serial per-kernel times (tools/pm_time.py, SYZGPU_PM_SERIAL=1) and the concurrent step
# (bench.py's step only). Usage (repo root, via gpurun): bash tools/gpu_ab_libs.sh TAG ENTRY...
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
  echo "== $i [$E]" | tee -a $OUT/ab.log
  env SYZGPU_LIB=$LIB $ENVS timeout -k 10 240 python -u -m pytest tests/test_gpu_raw.py -x -q --timeout 120 --timeout-method thread > $OUT/t$i.log 2>&1
  rc=$?; tail -1 $OUT/t$i.log | tee -a $OUT/ab.log; [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
  env SYZGPU_LIB=$LIB $ENVS SYZGPU_PM_SERIAL=1 timeout -k 10 120 python3 tools/pm_time.py > $OUT/pm$i.log 2>&1
  rc=$?; grep step_ms $OUT/pm$i.log | tee -a $OUT/ab.log; [ $rc -eq 0 ] || { echo "pm rc=$rc"; exit $rc; }
  env SYZGPU_LIB=$LIB $ENVS timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 3 --novelty 0 --text 0 --hub 0 \
      --analytics 0 --append 0 --store 0 --cooccurrence 0 --cpu-baseline 0 > $OUT/b$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 $OUT/b$i.log; exit $rc; }
  python3 -c "
import json
d=json.loads([l for l in open('$OUT/b$i.log') if l.startswith('{')][-1])
print('step', d['ms_per_step'], {k: v for k, v in list(d['kernels_ms_per_step_serialized_pass'].items())[:8]})" | tee -a $OUT/ab.log
done
