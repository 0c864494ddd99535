#!/bin/bash
# HBM traffic of the bench's kernels from rocprofv3 PMC counters, one counter set per pass
# (FETCH_SIZE and WRITE_SIZE cannot share a pass: MI355X_MICROARCH.md "rocprofv3 PMC slots").
# Usage (repo root, through gpurun): bash tools/gpu_pmc.sh TAG
set -o pipefail
TAG=${1:-pmc}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d $OUT/$C -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --profile 0 --novelty 0 --text 0 \
      --hub 0 --analytics 0 --append 0 --store 0 --cooccurrence 0 --setops 0 --canonicalize 0 --layout-change 0 > $OUT/$C.log 2>&1
  rc=$?; echo "$C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 $R/tools/pmc_traffic.py $OUT $OUT/pmc_traffic.json
