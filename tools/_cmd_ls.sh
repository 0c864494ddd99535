set -o pipefail
OUT=gpurun_out/r06_ls; mkdir -p $OUT; export TMPDIR=/tmp
SYZGPU_LIB=$GRAFT_REPO_ROOT/syzkaller_amd/libsyzgpu_ls512.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gosort.py tests/test_gpu_parity.py -k "gosort or sort or minimize" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_exp.sh r06_ls base ls512 base ls512
