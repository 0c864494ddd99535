set -o pipefail
OUT=gpurun_out/r06_xcd; mkdir -p $OUT; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
SYZGPU_LIB=$R/syzkaller_amd/libsyzgpu_xcd.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_raw.py tests/test_gpu_parity.py tests/test_gpu_novelty.py -k "minimize or raw or novelty" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_exp.sh r06_xcd base xcd base xcd || exit $?
cd /tmp
for L in base xcd; do
  LIB=$R/syzkaller_amd/libsyzgpu.so; [ $L = xcd ] && LIB=$R/syzkaller_amd/libsyzgpu_xcd.so
  SYZGPU_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w_$L -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --profile 0 --novelty 0 --text 0 \
      --hub 0 --analytics 0 --append 0 --store 0 --cooccurrence 0 --setops 0 --canonicalize 0 --layout-change 0 > $OUT/w_$L.log 2>&1
  rc=$?; echo "pmc $L rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd $R
python3 - <<'PY'
import csv, glob
from collections import defaultdict
for L in ['base','xcd']:
    acc=defaultdict(list)
    for f in glob.glob('gpurun_out/r06_xcd/w_%s/**/*counter_collection.csv' % L, recursive=True):
        for row in csv.DictReader(open(f)):
            acc[row['Kernel_Name'].split('(')[0][-30:]].append(float(row['Counter_Value']))
    for k,v in acc.items():
        if 'k_slab' in k or 'smin' in k: print(L, k, len(v), 'KiB/launch %.0f' % (sum(v)/len(v)))
PY
