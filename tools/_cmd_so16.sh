set -o pipefail
OUT=gpurun_out/r06_so16; mkdir -p $OUT; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
SYZGPU_LIB=$R/syzkaller_amd/libsyzgpu_so16.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "setop" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for v in base so16 base so16; do
  L=$R/syzkaller_amd/libsyzgpu.so; [ $v = so16 ] && L=$R/syzkaller_amd/libsyzgpu_so16.so
  SYZGPU_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-baseline 0 --store 0 --text 0 --novelty 0 \
    --canonicalize 0 --setops 1 --hub 0 --analytics 0 --append 0 --cooccurrence 0 --layout-change 0 > $OUT/b.json 2> $OUT/b.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/b.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('$OUT/b.json'))
print('$v', [(k, v['ms_per_batch'], v['kernels_ms'], v['roofline']['frac']) for k,v in d['setops_triage']['ops'].items()])" | tee -a $OUT/ab.log
done
