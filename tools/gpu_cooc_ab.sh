#!/bin/bash
# Co-occurrence A/B on the GPU box: for each GEMM form (SYZGPU_CO_FORM), the parity tests, then the
# bench leg under several forced K splits ("d" = the library's default split); FORMS entries are
# form or form.prefetch (e.g. "0.2").
set -o pipefail
out=gpurun_out/${1:-cooc_ab}; mkdir -p $out
for fp in ${FORMS:-0}; do
  form=$fp
  export SYZGPU_CO_FORM=${fp%%.*} SYZGPU_CO_PF=${fp#*.}
  [ "$SYZGPU_CO_PF" = "$fp" ] && SYZGPU_CO_PF=
  timeout -k 10 300 python -u -m pytest tests/test_gpu_cooccur.py -q -x --timeout 200 --timeout-method thread > $out/pytest_$form.log 2>&1
  rc=$?; echo "form $form: $(tail -1 $out/pytest_$form.log)"; [ $rc -eq 0 ] || exit $rc
  for ks in ${KSLIST:-d 16 24 32}; do
    k=$ks; [ "$ks" = d ] && k=
    SYZGPU_CO_KS=$k timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-baseline 0 --store 0 --text 0 --novelty 0 --hub 0 --analytics 0 --append 0 > $out/b_${form}_$ks.json 2> $out/b_${form}_$ks.err || exit $?
    python - $out/b_${form}_$ks.json "$form" "$ks" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("call_cooccurrence") or {}
print("form=%s ks=%s" % (sys.argv[2], sys.argv[3]), c.get("ms"), c.get("kernels_ms"), (c.get("roofline") or {}).get("frac"))
PY
  done
done
