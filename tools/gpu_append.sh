#!/bin/bash
# The resident corpus lifecycle: its GPU tests, then the bench's store + manager-cycle legs alone.
# Usage (through gpurun): bash tools/gpu_append.sh TAG [VAR=value ...]
set -o pipefail
TAG=${1:-app}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_append.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert" $OUT/pytest.log | head -20; exit $rc; }
env "$@" timeout -k 10 300 python3 -u bench.py --steps 4 --warmup 1 --cpu-baseline 0 --text 0 --novelty 0 --hub 0 --analytics 0 --cooccurrence 0 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "
import json,sys
r=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('step', r['ms_per_step'], 'store', r['store_reuse']['minimize_ms'], r['store_reuse']['ingest_s'])
for c in r['manager_cycle']['cycles']: print(c)
"
