#!/bin/bash
# set-op leg timing per library variant (dev tooling). Usage (via gpurun): bash tools/gpu_so_ab.sh TAG LIBTAG...
# ("base" = syzkaller_amd/libsyzgpu.so, else syzkaller_amd/libsyzgpu_LIBTAG.so)
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for rep in 1 2; do
for L in "$@"; do
  LIB=$GRAFT_REPO_ROOT/syzkaller_amd/libsyzgpu.so; [ $L != base ] && LIB=$GRAFT_REPO_ROOT/syzkaller_amd/libsyzgpu_$L.so
  SYZGPU_LIB=$LIB timeout -k 10 300 python -u tools/leg_time.py setops --steps 6 --cpu-baseline 0 > $OUT/so_$L.log 2>&1 || { tail -3 $OUT/so_$L.log; exit 1; }
  python3 - $OUT/so_$L.log "$L" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], {k: (v["ms_per_batch"], v["kernels_ms"].get("setop_merge")) for k, v in d["ops"].items()})
PY
done
done
