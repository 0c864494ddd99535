set -o pipefail
mkdir -p gpurun_out/r06_thr
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_threads.py tests/test_multi.py tests/test_gpu_raw.py tests/test_abi.py > gpurun_out/r06_thr/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06_thr/tests.log; exit $rc
