#!/bin/bash
set -o pipefail
bash tools/gpu_so.sh e6 base sc4 so128x16 so128x16sc4 so256x8 so64x16 || exit $?
cd /tmp
PM_K=2 PM_W=2 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/e6/kt -o run -- python3 $GRAFT_REPO_ROOT/tools/pm_time.py > $GRAFT_REPO_ROOT/gpurun_out/e6/kt.log 2>&1
