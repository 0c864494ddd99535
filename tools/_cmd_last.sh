set -o pipefail
mkdir -p gpurun_out/r06_last
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_threads.py tests/test_gpu_raw.py tests/test_gpu_gosort.py tests/test_multi.py > gpurun_out/r06_last/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06_last/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_last/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r06_last/smoke.log; exit $rc
