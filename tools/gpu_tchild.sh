set -o pipefail
mkdir -p gpurun_out/tchild
for v in 4096 2048; do
  SYZGPU_GS_T_CHILD=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_gosort.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tchild/t_$v.log 2>&1 || { tail -20 gpurun_out/tchild/t_$v.log; exit 1; }
  tail -1 gpurun_out/tchild/t_$v.log
done
bash tools/gpu_sweep_env.sh tchild SYZGPU_GS_T_CHILD 8192 4096 2048 1024 -- --novelty 0 --text 0 --hub 0 --analytics 0
