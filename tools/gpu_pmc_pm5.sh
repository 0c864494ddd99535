#!/bin/bash
# PMC passes over the raw minimize job alone (tools/pm_time.py, serialized kernels): two SQ counter
# sets and the HBM traffic (FETCH_SIZE / WRITE_SIZE), one set per pass, then per-kernel means.
# Usage (repo root, through gpurun): bash tools/gpu_pmc_pm5.sh TAG
set -o pipefail
TAG=${1:-pmcpm}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU" \
         "SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_SALU" \
         FETCH_SIZE WRITE_SIZE; do
  i=$((i+1)); D=$OUT/p$i; [ "$C" = FETCH_SIZE ] && D=$OUT/FETCH_SIZE; [ "$C" = WRITE_SIZE ] && D=$OUT/WRITE_SIZE
  SYZGPU_PM_SERIAL=1 PM_K=2 PM_W=1 timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $D -o run -- \
    python3 $R/tools/pm_time.py > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 $R/tools/pmc_traffic.py $OUT $OUT/pmc_traffic.json
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, json
from collections import defaultdict
d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "p[12]", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0][-40:]
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
res = {}
for k, c in sorted(acc.items()):
    if "syz" not in k:
        continue
    res[k] = {n: round(sum(v) / len(v)) for n, v in sorted(c.items())}
    print(k, res[k])
json.dump(res, open(os.path.join(d, "sq.json"), "w"), indent=1)
t = json.load(open(os.path.join(d, "pmc_traffic.json")))
for k, v in t["kernels"].items():
    print(k, v)
PY
