#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no HIP events in the step), then the per-step
# timeline. Usage (repo root, through gpurun): bash tools/gpu_trace.sh TAG [bench args...]
set -o pipefail
TAG=${1:-trace}; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 $R/bench.py --cpu-baseline 0 --raw-steps 0 --profile 0 --steps 5 --warmup 2 "$@" > $OUT/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 $R/tools/trace_summary.py $OUT/prof/run_kernel_trace.csv k_gs_init > $OUT/timeline.txt 2>&1
tail -40 $OUT/timeline.txt
