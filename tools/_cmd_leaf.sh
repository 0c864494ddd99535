set -o pipefail
OUT=gpurun_out/r06_leaf; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gosort.py tests/test_gpu_parity.py tests/test_gpu_raw.py -k "order or leaf or minimize or raw" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_exp.sh r06_leaf base
