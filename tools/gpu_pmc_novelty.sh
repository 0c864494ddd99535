#!/bin/bash
# HBM traffic of the config-3 novelty kernels (FETCH_SIZE, WRITE_SIZE: one rocprofv3 pass each).
# Usage (repo root, through gpurun): bash tools/gpu_pmc_novelty.sh TAG
set -o pipefail
TAG=${1:-pmcnov}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $OUT/$C -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --cpu-baseline 0 --raw-steps 0 --profile 0 --text 0 --hub 0 \
      --analytics 0 --novelty-cpu-sample 10 > $OUT/$C.log 2>&1
  rc=$?; echo "$C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - $OUT <<'PY'
import csv, glob, json, os, sys
out = sys.argv[1]
res = {}
for C in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(os.path.join(out, C, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            n = row.get("Kernel_Name", "")
            if row.get("Counter_Name") != C or "k_kt_" not in n:
                continue
            k = n.split("(")[0].replace("syz::", "")
            res.setdefault(k, {}).setdefault(C, []).append(float(row["Counter_Value"]))
summ = {k: {C: sum(v) / len(v) * 1024 for C, v in d.items()} for k, d in res.items()}
json.dump(summ, open(os.path.join(out, "novelty_pmc.json"), "w"), indent=1)
print(json.dumps(summ))
PY
