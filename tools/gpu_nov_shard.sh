#!/bin/bash
# Rehearsal of bench.py's N>1 novelty leg on one GPU: N=1 and a 2-rank gloo run with both ranks on GPU 0
# (reduced sizes); the two novelty_config3.new_covers must agree. Usage: bash tools/gpu_nov_shard.sh TAG
set -o pipefail
TAG=${1:-novsh}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
A="--steps 4 --warmup 1 --progs-per-gpu 100000 --novelty-covers 200000 --cpu-baseline 0 --store 0 --text 0 --hub 0 --analytics 0 --append 0 --cooccurrence 0 --novelty-wide 0"
timeout -k 10 300 python3 -u bench.py $A > $OUT/n1.json 2> $OUT/n1.err || { tail -5 $OUT/n1.err; exit 1; }
SYZ_BENCH_BACKEND=gloo SYZ_BENCH_SAME_DEVICE=1 timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 $A > $OUT/n2.json 2> $OUT/n2.err || { tail -20 $OUT/n2.err; exit 1; }
python3 - $OUT <<'PY'
import json, sys
o = sys.argv[1]
a = json.loads(open(o + "/n1.json").read().strip().splitlines()[-1])["novelty_config3"]
b = json.loads(open(o + "/n2.json").read().strip().splitlines()[-1])["novelty_config3"]
print("N=1", {k: a[k] for k in ("ms_per_batch", "new_covers", "maxcover_out_pcs")})
print("N=2", {k: b[k] for k in ("ms_per_batch", "new_covers", "maxcover_out_pcs", "exchange_bytes_per_batch")})
assert a["new_covers"] == b["new_covers"] and a["maxcover_out_pcs"] == b["maxcover_out_pcs"], "mismatch"
print("sharded novelty matches")
PY
