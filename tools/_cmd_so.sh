set -o pipefail
OUT=gpurun_out/r06_so; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "setop" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for v in base gap lbm32; do
  L=syzkaller_amd/libsyzgpu.so; E=""
  [ $v = gap ] && { L=syzkaller_amd/libsyzgpu_sogap.so; E="SYZGPU_SO_GAP=1"; }
  [ $v = lbm32 ] && L=syzkaller_amd/libsyzgpu_lbm32.so
  env SYZGPU_LIB=$L $E timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-baseline 0 --store 0 --text 0 --novelty 0 \
    --canonicalize 0 --setops 1 --hub 0 --analytics 0 --append 0 --cooccurrence 0 --layout-change 0 > $OUT/bench_$v.json 2> $OUT/bench_$v.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/bench_$v.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_$v.json'))
for k,v in d['setops_triage']['ops'].items(): print('$v', k, v['ms_per_batch'], v['kernels_ms'], v['roofline']['frac'])"
done
