#!/bin/bash
# Co-occurrence A/B on the GPU box: parity tests, then the bench leg under several forced K splits.
set -o pipefail
out=gpurun_out/${1:-cooc_ab}; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_cooccur.py -q -x --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for ks in ${KSLIST:-"" 8 16 24 32 19}; do
  SYZGPU_CO_KS=$ks timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-baseline 0 --store 0 --text 0 --novelty 0 --hub 0 --analytics 0 --append 0 > $out/b_$ks.json 2> $out/b_$ks.err || exit $?
  python - $out/b_$ks.json "$ks" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("call_cooccurrence") or {}
print("ks=%s" % sys.argv[2], c.get("ms"), c.get("kernels_ms"), (c.get("roofline") or {}).get("frac"))
PY
done
