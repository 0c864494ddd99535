set -o pipefail
mkdir -p gpurun_out/r06_o
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_raw.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_multi.py -k "minimize or raw or config4 or multi" > gpurun_out/r06_o/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06_o/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_exp.sh r06_o base wwp
