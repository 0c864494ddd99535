#!/bin/bash
# A/B of the config-3 novelty leg (default + wide span) under env variants, one after another.
# Usage (through gpurun): bash tools/gpu_nov_ab.sh TAG "VAR=v VAR2=w" "VAR=x" ...  ("base" = no vars)
set -o pipefail
TAG=${1:-novab}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i + 1))
  [ "$v" = "base" ] && v=""
  env $v timeout -k 10 240 python3 -u tools/nov_bench.py 4 > $OUT/v$i.log 2>&1 || { echo "variant $i failed"; tail -5 $OUT/v$i.log; exit 1; }
  python3 - "$v" $OUT/v$i.log <<'PY'
import json, sys
r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
w = r.get("wide_span", {})
print(repr(sys.argv[1]), "default", r["ms_per_batch"], r["kernels_ms_per_batch"], "| wide", w.get("ms_per_batch"), w.get("kernels_ms_per_batch"))
PY
done
