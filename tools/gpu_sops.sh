#!/bin/bash
# Set algebra on the GPU: the parity tests, then the bench's setops_triage leg alone. Usage: bash tools/gpu_sops.sh TAG
set -o pipefail
TAG=${1:-sops}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $OUT/pytest.log | head; exit $rc; }
timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --cpu-baseline 0 --store 0 --text 0 --novelty 0 --hub 0 \
  --analytics 0 --append 0 --cooccurrence 0 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json; r=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(r['ms_per_step'], json.dumps({k: v['ms_per_batch'] for k, v in r['setops_triage']['ops'].items()}))"
