#!/bin/bash
# Kernel stats of one bench leg (dev tooling). Usage: LEG=novelty bash tools/gpu_leg_prof.sh TAG
set -o pipefail
TAG=${1:-leg}
LEG=${LEG:-novelty}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --cpu-baseline 0 --profile 0"
for l in store text novelty hub analytics append cooccurrence setops canonicalize; do
  [ "$l" = "$LEG" ] || ARGS="$ARGS --$l 0"
done
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 $R/bench.py $ARGS > $OUT/bench.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
    print("%-70s %6s %10.3f ms %9.1f us" % (r["Name"][:70], r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e3))
PY
