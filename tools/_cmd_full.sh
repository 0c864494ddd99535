set -o pipefail
mkdir -p gpurun_out/r06_full
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -x > gpurun_out/r06_full/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r06_full/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_full/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/r06_full/smoke.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_final6.sh r06_final5 && bash tools/gpu_configs.sh r06_configs6
