#!/bin/bash
# A/B of the persistent gosort rounds' grid size against the graph path
set -o pipefail
mkdir -p gpurun_out/ab
for cfg in "SYZGPU_GR_PERSIST=0" "SYZGPU_GR_PERSIST=1 SYZGPU_GR_PGRID=64" "SYZGPU_GR_PERSIST=1 SYZGPU_GR_PGRID=128" "SYZGPU_GR_PERSIST=1 SYZGPU_GR_PGRID=256"; do
  env $cfg timeout -k 10 200 python -u bench.py --novelty 0 --text 0 --hub 0 --analytics 0 --raw-steps 0 --cpu-baseline 0 > gpurun_out/ab/b.log 2>&1 || { tail -5 gpurun_out/ab/b.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/ab/b.log') if l.startswith('{')][-1])
k=d['kernels_ms_per_step_serialized_pass']
print('$cfg', d['ms_per_step'], 'level', k['gosort_level'], 'lds_small', k['gosort_lds_small'], 'vmin', k['vec_min'])"
done
