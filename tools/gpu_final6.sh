#!/bin/bash
# Round-6 closing evidence on one GPU: the default bench line (every leg), a rocprofv3 kernel-trace
# summary + trace of the headline step alone (-> the step timeline), its FETCH_SIZE / WRITE_SIZE passes and
# one SQ-counter pass. Usage (through gpurun, repo root): bash tools/gpu_final6.sh TAG
set -o pipefail
TAG=${1:-final6}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
STEP="--cpu-baseline 0 --store 0 --text 0 --novelty 0 --hub 0 --analytics 0 --append 0 --cooccurrence 0 --setops 0 --canonicalize 0 --layout-change 0"
timeout -k 10 600 python3 -u $R/bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 $STEP > $OUT/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/prof_bench.log; exit $rc; }
cd $R && python3 tools/timeline.py $OUT/prof > $OUT/step_timeline.txt 2>&1; head -3 $OUT/step_timeline.txt
bash tools/gpu_pmc.sh $TAG/pmc || exit $?
BENCH_ARGS="$STEP" bash tools/gpu_pmc_sq.sh $TAG/sq
