set -o pipefail
mkdir -p gpurun_out/r03_rgdbg
for D in 0 16 32 64; do
  SYZGPU_RG_DBG=$D SYZGPU_PM_SERIAL=1 timeout -k 10 120 python3 tools/pm_time.py >> gpurun_out/r03_rgdbg/pm.log 2>&1 || exit 1
done
grep step_ms gpurun_out/r03_rgdbg/pm.log
