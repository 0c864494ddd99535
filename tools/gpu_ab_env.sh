#!/bin/bash
# A/B of one environment knob on the bench's side legs. Usage (repo root, through gpurun):
#   bash tools/gpu_ab_env.sh TAG "bench args" "ENV=a" "ENV=b" ...   (prints each leg's kernel times)
set -o pipefail
TAG=$1; ARGS=$2; shift 2
mkdir -p gpurun_out/$TAG
for cfg in "$@"; do
  env $cfg timeout -k 10 240 python -u bench.py $ARGS > gpurun_out/$TAG/b.log 2>&1 || { tail -5 gpurun_out/$TAG/b.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/$TAG/b.log') if l.startswith('{')][-1])
out={'step': d['ms_per_step']}
for k in ('minimize_corpus_tail','novelty_config3','cover_analytics','hub_ingest_config5'):
    if d.get(k): out[k]=(d[k].get('ms', d[k].get('ms_per_batch')), d[k].get('kernels_ms', d[k].get('kernels_ms_per_batch')))
print('$cfg', json.dumps(out))"
done
