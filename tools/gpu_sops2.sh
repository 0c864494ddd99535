#!/bin/bash
# One short GPU call: set-op / canonicalize parity tests, then the bench's set-op and canonicalize legs
# at the default tile-walk grid and a smaller one.
set -o pipefail
TAG=${1:-sops2}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
LEGS="--steps 3 --warmup 1 --cpu-baseline 0 --store 0 --text 0 --novelty 0 --hub 0 --analytics 0 --append 0 --cooccurrence 0"
for e in "X=0"; do
  env $e timeout -k 10 300 python3 bench.py $LEGS > $OUT/bench_$e.json 2> $OUT/bench_$e.err || exit 1
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], {k:(v['ms_per_batch'], v.get('kernels_ms')) for k,v in d['setops_triage']['ops'].items()}, 'canon', d['canonicalize_raw_covers']['ms_per_batch'])" $OUT/bench_$e.json $e
done
