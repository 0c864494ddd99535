#!/bin/bash
# Two SQ-counter passes over the bench's novelty leg (dev tooling). Usage: bash tools/gpu_pmc_nov.sh TAG
set -o pipefail
TAG=${1:-pmc_nov}
export BENCH_ARGS="--store 0 --text 0 --setops 0 --canonicalize 0 --hub 0 --analytics 0 --append 0 --cooccurrence 0"
bash tools/gpu_pmc_sq.sh ${TAG}_a || exit $?
CTR="SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM" \
  bash tools/gpu_pmc_sq.sh ${TAG}_b
