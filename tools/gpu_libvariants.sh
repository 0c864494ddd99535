#!/bin/bash
# A/B of compile-time variants: for each syzkaller_amd/libsyzgpu_<tag>.so given, the gosort tests and the
# headline bench line with SYZGPU_LIB pointing at it. Usage: bash tools/gpu_libvariants.sh tag1 tag2 ...
set -o pipefail
mkdir -p gpurun_out/variants
for t in "$@"; do
  lib=$GRAFT_REPO_ROOT/syzkaller_amd/libsyzgpu_$t.so
  SYZGPU_LIB=$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_gosort.py -x -q --timeout 120 --timeout-method thread > gpurun_out/variants/t_$t.log 2>&1 || { echo "$t tests failed"; tail -5 gpurun_out/variants/t_$t.log; exit 1; }
  SYZGPU_LIB=$lib timeout -k 10 200 python -u bench.py --novelty 0 --text 0 --hub 0 --analytics 0 --raw-steps 0 --cpu-baseline 0 > gpurun_out/variants/b_$t.log 2>&1 || { tail -5 gpurun_out/variants/b_$t.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/variants/b_$t.log') if l.startswith('{')][-1])
k=d['kernels_ms_per_step_serialized_pass']
print('$t', d['ms_per_step'], 'gosort_level', k['gosort_level'], 'vec_min', k['vec_min'])"
done
