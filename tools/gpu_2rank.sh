#!/bin/bash
# Two-rank rehearsal of the N>1 bench on one GPU (dev tooling): bash tools/gpu_2rank.sh (via gpurun)
set -o pipefail
mkdir -p gpurun_out/r06_2rank
# the N>1 path rehearsed on one GPU: every rank on cuda:0, collectives over gloo (RCCL refuses two ranks on one device)
export SYZ_BENCH_SAME_DEVICE=1 SYZ_BENCH_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/r06_2rank/bench.json 2> gpurun_out/r06_2rank/bench.err
rc=$?; tail -3 gpurun_out/r06_2rank/bench.err; exit $rc
