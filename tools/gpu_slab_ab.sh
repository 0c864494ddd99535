#!/bin/bash
# A/B of library variants (tools/build_variant.sh) and environment settings on the raw minimize job
# (pm_time.py, serialized and concurrent), then SQ counter passes of the default library.
# Usage (through gpurun): bash tools/gpu_slab_ab.sh TAG [LIB[:VAR=val[,VAR=val]] ...]   (LIB base = default)
set -o pipefail
TAG=${1:-ab}; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for spec in base "$@"; do
  v=${spec%%:*}; envs=""; [ "$spec" != "$v" ] && envs=$(echo ${spec#*:} | tr ',' ' ')
  lib=$R/syzkaller_amd/libsyzgpu.so; [ $v = base ] || lib=$R/syzkaller_amd/libsyzgpu_$v.so
  for e in "SYZGPU_PM_SERIAL=1" "X=0"; do
    echo "== $spec $e" >> $OUT/pm.log
    env SYZGPU_LIB=$lib $envs $e timeout -k 10 120 python3 $R/tools/pm_time.py 2>&1 | grep -v amdgpu.ids >> $OUT/pm.log || { tail -5 $OUT/pm.log; exit 1; }
  done
done
cat $OUT/pm.log
[ -n "$NO_PMC" ] && exit 0
cd /tmp
i=0
for CTR in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM"; do
  i=$((i+1))
  SYZGPU_PM_SERIAL=1 PM_K=2 PM_W=1 timeout -s KILL 90 rocprofv3 --pmc $CTR --output-format csv -d $OUT/pmc$i -o run -- python3 $R/tools/pm_time.py > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, json
from collections import defaultdict
d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True):
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
PY
