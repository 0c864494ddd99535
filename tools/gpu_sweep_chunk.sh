#!/bin/bash
# bench line at several vec_min work-item sizes (SYZGPU_CHUNK_VECS), no side legs
set -o pipefail
mkdir -p gpurun_out/sweep
for cv in ${@:-32768 65536 131072}; do
  SYZGPU_CHUNK_VECS=$cv timeout -k 10 200 python -u bench.py --novelty 0 --text 0 --hub 0 --analytics 0 --raw-steps 0 \
    --cpu-baseline 0 > gpurun_out/sweep/cv_$cv.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/sweep/cv_$cv.log') if l.startswith('{')][-1])
print($cv, d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['kernels_ms_per_step_serialized_pass']['vec_min_small'])"
done
