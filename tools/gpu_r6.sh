#!/bin/bash
# Round-6 iteration run (dev tooling): the raw-minimize parity tests named by $TESTS (default: the raw
# pipeline and speculation tests), then the headline bench line with only the layout-change leg.
# Usage (repo root, via gpurun): TESTS="files" KEXPR="-k expression" bash tools/gpu_r6.sh TAG
set -o pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
T=${TESTS:-"tests/test_gpu_raw.py tests/test_gpu_parity.py"}
K=${KEXPR:-"minimize or raw or multi"}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread $T -k "$K" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline 0 --store 0 --text 0 --novelty 0 \
  --canonicalize 0 --setops 0 --hub 0 --analytics 0 --append 0 --cooccurrence 0 ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
print('ms_per_step', d['ms_per_step'], 'roof', d['roofline'] and d['roofline']['frac'], 'job', d['job'])
print('layout_change', d['layout_change'])
print({k: v for k, v in list(d['kernels_ms_per_step_serialized_pass'].items())[:12]})"
