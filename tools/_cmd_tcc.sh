set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r06_tcc; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $OUT/pmc -o run -- \
  python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --profile 0 --novelty 0 --text 0 \
    --hub 0 --analytics 0 --append 0 --store 0 --cooccurrence 0 --setops 0 --canonicalize 0 --layout-change 0 > $OUT/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R
python3 - <<'PY'
import csv, glob
from collections import defaultdict
acc=defaultdict(lambda: defaultdict(list))
for f in glob.glob('gpurun_out/r06_tcc/pmc/**/*counter_collection.csv', recursive=True):
    for row in csv.DictReader(open(f)):
        k=row['Kernel_Name'].split('(')[0][-32:]
        acc[k][row['Counter_Name']].append(float(row['Counter_Value']))
for k,c in acc.items():
    if any(x in k for x in ('k_slab','smin','k_ls_sort','k_gr_')):
        print(k, {n: round(sum(v)/len(v)) for n,v in c.items()})
PY
