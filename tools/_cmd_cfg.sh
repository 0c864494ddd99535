set -o pipefail
mkdir -p gpurun_out/r06_cfgt
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_threads.py tests/test_gpu_raw.py tests/test_gpu_configs.py > gpurun_out/r06_cfgt/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06_cfgt/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_configs.sh r06_configs4
