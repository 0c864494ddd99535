#!/bin/bash
# Kernel stats of the bench's canonicalize leg (dev tooling). Usage: bash tools/gpu_canon_prof.sh TAG
set -o pipefail
TAG=${1:-canon}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --profile 0 --store 0 --text 0 --novelty 0 --hub 0 \
    --analytics 0 --append 0 --cooccurrence 0 --setops 0 > $OUT/bench.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print("%-70s %6s %10.3f ms %9.1f us" % (r["Name"][:70], r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e3))
PY
