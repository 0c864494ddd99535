#!/bin/bash
# The headline step at each BASELINE.json config on one GPU (BASELINE.md's table), with the
# single-core and multi-core CPU restatement on the same corpus. Usage: bash tools/gpu_configs.sh TAG
set -o pipefail
TAG=${1:-cfg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
LEGS="--text 0 --novelty 0 --hub 0 --analytics 0 --append 0 --store 1 --cooccurrence 0 --setops 0 --canonicalize 0"
run() {  # name, args...
  n=$1; shift
  timeout -k 10 600 python -u bench.py $LEGS "$@" > $OUT/$n.log 2>&1 || { echo "$n failed"; tail -5 $OUT/$n.log; exit 1; }
  grep '^{' $OUT/$n.log | tail -1 > $OUT/$n.json
  python3 -c "
import json; d=json.load(open('$OUT/$n.json')); c=d.get('cpu_baseline') or {}
print('$n', d['ms_per_step'], 'ms', round(d['value']/1e6,2), 'Mprogs/s', 'cpu1', c.get('value'), 'cpuN', (c.get('multi_thread') or {}).get('value'))"
}
run config1 --progs-per-gpu 10000 --npcs 50000 --steps 20 --warmup 3
run config2 --progs-per-gpu 100000 --npcs 500000 --steps 20 --warmup 3
run config4 --progs-per-gpu 1000000 --npcs 2000000 --steps 10 --warmup 3
run config5 --progs-per-gpu 8000000 --npcs 2000000 --steps 5 --warmup 2 --cpu-sample 1000000
