#!/bin/bash
# Per-rank rehearsal of the weak-scaling job on one GPU: rank r's shard of a W-rank corpus.
# Usage (repo root, through gpurun): bash tools/gpu_emulate.sh TAG W:r [W:r ...]
set -o pipefail
TAG=${1:-emu}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for WR in "$@"; do
  LOG=$OUT/emu_${WR/:/_}.log
  timeout -k 10 240 python -u bench.py --cpu-baseline 0 --store 0 --text 0 --novelty 0 --hub 0 --analytics 0 --append 0 --cooccurrence 0 --emulate $WR > $LOG 2>&1
  rc=$?; echo "$WR rc=$rc"; [ $rc -eq 0 ] || { tail -5 $LOG; exit $rc; }
  grep -o '"ms_per_step": [0-9.]*\|"max_rank_load_share": [0-9.]*\|"total_progs": [0-9]*' $LOG | tr '\n' ' '; echo
done
