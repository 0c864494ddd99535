set -o pipefail
OUT=gpurun_out/r06_f2; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_raw.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_multi.py -k "minimize or raw or config or multi" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_final6.sh r06_final2
