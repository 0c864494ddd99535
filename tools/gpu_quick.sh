#!/bin/bash
# Quick GPU-box pass: selected tests (pytest -k expr) then one bench line.
# Usage: bash tools/gpu_quick.sh TAG 'pytest-k-expr' [bench args...]
set -o pipefail
TAG=${1:-quick}; K=${2:-gosort}; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; exit $rc; }
timeout -k 10 300 python -u bench.py --cpu-baseline 0 "$@" > $OUT/bench.log 2>&1
rc=$?; tail -c 2500 $OUT/bench.log; exit $rc
