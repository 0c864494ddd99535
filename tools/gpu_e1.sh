timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_append.py -k "multirank or failed_growth or gate_vs" > gpurun_out/e1_tests.log 2>&1; echo "tests rc=$?"; tail -5 gpurun_out/e1_tests.log
bash tools/gpu_exp.sh e1 base mident "base|SYZGPU_RG_DBG=16" "base|SYZGPU_RG_DBG=32"
