set -o pipefail
OUT=gpurun_out/r06_px; mkdir -p $OUT; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
SYZGPU_LIB=$R/syzkaller_amd/libsyzgpu_px16.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_raw.py tests/test_gpu_parity.py tests/test_gpu_novelty.py -k "minimize or raw or windows" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_exp.sh r06_px base px16 px64 base px16 px64
