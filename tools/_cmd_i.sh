set -o pipefail
mkdir -p gpurun_out/r06_i
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_raw.py tests/test_gpu_parity.py tests/test_gpu_configs.py -k "minimize or raw or config4" > gpurun_out/r06_i/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06_i/tests.log; [ $rc -eq 0 ] || exit $rc
SYZGPU_PM_SERIAL=1 timeout -k 10 200 python -u tools/smin_stats.py > gpurun_out/r06_i/stats.log 2>&1 || exit 1
tail -3 gpurun_out/r06_i/stats.log
bash tools/gpu_exp.sh r06_i base
