#!/bin/bash
# One GPU call for a round checkpoint: the full -m gpu suite, then the raw-pipeline A/B variants and SQ
# counters (tools/gpu_slab_ab.sh), then a short bench line. Stops at the first failing step.
# Usage (through gpurun): bash tools/gpu_check_all.sh TAG [variants for gpu_slab_ab.sh ...]
set -o pipefail
TAG=${1:-check}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; exit $rc; }
NO_PMC=${NO_PMC:-} bash tools/gpu_slab_ab.sh $TAG "$@" > $OUT/ab.log 2>&1
rc=$?; tail -30 $OUT/ab.log | cut -c1-400; [ $rc -eq 0 ] || { echo "ab failed rc=$rc"; exit $rc; }
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 > $OUT/bench.log 2>&1
rc=$?; tail -c 3000 $OUT/bench.log; exit $rc
