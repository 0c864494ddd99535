#!/bin/bash
# Config-3 novelty A/B: tools/nov_bench.py under each "VAR=value ..." setting given, then one SQ-counter
# pass and the FETCH/WRITE passes of the default. Usage (repo root, via gpurun):
#   bash tools/gpu_nov_ab.sh TAG "SYZGPU_NW_DBG=1" "SYZGPU_NW_DBG=2" ...
set -o pipefail
TAG=${1:-novab}; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for SET in "" "$@"; do
  i=$((i+1))
  echo "== [$SET]" | tee -a $OUT/ab.log
  env $SET timeout -k 10 180 python3 -u tools/nov_bench.py 4 > $OUT/ab$i.json 2> $OUT/ab$i.err
  rc=$?; [ $rc -eq 0 ] || { echo "run $i rc=$rc"; tail -5 $OUT/ab$i.err; exit $rc; }
  python3 -c "import json,sys; d=json.load(open('$OUT/ab$i.json')); print(d['ms_per_batch'], d['kernels_ms_per_batch'])" | tee -a $OUT/ab.log
done
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/tools/nov_bench.py 2 > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -30
[ -n "$NOPMC" ] && exit 0
p=0
for CTR in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  p=$((p+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d $OUT/pmc$p -o run -- python3 $R/tools/nov_bench.py 1 > $OUT/pmc$p.log 2>&1
  rc=$?; echo "pmc pass $p rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0][-30:]
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, c in sorted(acc.items()):
    if "k_nw" in k or "part3" in k or "grp" in k:
        print(k, {n: round(sum(v) / len(v)) for n, v in sorted(c.items())})
PY
