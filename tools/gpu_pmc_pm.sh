#!/bin/bash
# PMC passes over the raw minimize job alone (tools/pm_time.py, serial P then sort then M): one rocprofv3
# run per counter set (sets within the per-block limits), then per-kernel means.
# Usage (repo root, through gpurun): bash tools/gpu_pmc_pm.sh TAG [VAR=value ...]
set -o pipefail
TAG=${1:-pmcpm}; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for CTR in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU" \
           "FETCH_SIZE TA_BUSY_avr TA_BUSY_max" "WRITE_SIZE"; do
  i=$((i+1))
  env "$@" SYZGPU_PM_SERIAL=1 PM_K=2 timeout -s KILL 90 rocprofv3 --pmc $CTR --output-format csv -d $OUT/p$i -o run -- \
    python3 $R/tools/pm_time.py > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0][-44:]
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, c in sorted(acc.items()):
    if "syz" not in k:
        continue
    print(k, {n: round(sum(v) / len(v)) for n, v in sorted(c.items())})
PY
