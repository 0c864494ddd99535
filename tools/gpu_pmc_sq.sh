#!/bin/bash
# One SQ-counter pass (wave time split into parked / issue-stalled / issuing, LDS bank conflicts) over a
# short bench run, then per-kernel means. Usage (repo root, through gpurun): bash tools/gpu_pmc_sq.sh TAG
# (CTR overrides the counter set, BENCH_ARGS adds bench flags)
set -o pipefail
TAG=${1:-sq}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
CTR=${CTR:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU"}
timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d $OUT/pmc -o run -- \
  python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --profile 0 ${BENCH_ARGS:-} > $OUT/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - "$OUT" <<'EOF'
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "pmc", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0][-40:]
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, c in sorted(acc.items()):
    if not k.strip().startswith(("syz", "void syz")):
        continue
    print(k, {n: round(sum(v) / len(v)) for n, v in sorted(c.items())})
EOF
