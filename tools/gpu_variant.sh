#!/bin/bash
# One GPU call for a library variant: its raw-minimize parity tests (configs, raw pipeline, novelty),
# then the A/B of the default library and the given specs with SQ counters (tools/gpu_slab_ab.sh).
# Usage (through gpurun): bash tools/gpu_variant.sh TAG VARIANT [more specs for gpu_slab_ab.sh ...]
set -o pipefail
TAG=${1:-var}; V=$2; shift 2
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
SYZGPU_LIB=$R/syzkaller_amd/libsyzgpu_$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_raw.py tests/test_gpu_configs.py tests/test_gpu_novelty.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_slab_ab.sh $TAG $V "$@" > $OUT/ab.log 2>&1
rc=$?; tail -40 $OUT/ab.log | cut -c1-300; exit $rc
