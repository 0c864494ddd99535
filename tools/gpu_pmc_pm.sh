#!/bin/bash
# SQ-counter passes over the raw minimize job (tools/pm_time.py, serial streams), per-kernel means.
# Usage (repo root, through gpurun): bash tools/gpu_pmc_pm.sh TAG
set -o pipefail
TAG=${1:-pmc}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp SYZGPU_PM_SERIAL=1 SYZGPU_GS_NOFORK=1 PM_N=${PM_N:-1000000} SYZGPU_PART=${SYZGPU_PART:-1}
cd /tmp
i=0
for CTR in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d $OUT/pmc$i -o run -- python3 $R/tools/pm_time.py > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
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
    if "pmin" in k or "part" in k or "tiles" in k:
        print(k, {n: round(sum(v) / len(v)) for n, v in sorted(c.items())})
PY
