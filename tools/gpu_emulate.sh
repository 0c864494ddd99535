#!/bin/bash
# Per-rank rehearsal of the weak-scaling job on one GPU: rank r's shard of a W-rank corpus.
# Usage (repo root, through gpurun): bash tools/gpu_emulate.sh TAG W:r [W:r ...]
set -o pipefail
TAG=${1:-emu}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for WR in "$@"; do
  LOG=$OUT/emu_${WR/:/_}.log
  timeout -k 10 240 python -u bench.py --cpu-baseline 0 --store 0 --text 0 --novelty 0 --hub 0 --analytics 0 --append 0 --cooccurrence 0 --setops 0 --canonicalize 0 --emulate $WR > $LOG 2>&1
  rc=$?; echo "$WR rc=$rc"; [ $rc -eq 0 ] || { tail -5 $LOG; exit $rc; }
  python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=r[\"kernels_ms_per_step_serialized_pass\"]; print(r[\"ms_per_step\"], {x: k[x] for x in k if x.startswith(\"gosort\") or x in (\"m_big\", \"m_small\", \"k_region\")}, r[\"config\"][\"split_groups\"])" $LOG
done
