set -o pipefail
OUT=gpurun_out/r06_c2c; mkdir -p $OUT; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LEGS="--text 0 --novelty 0 --hub 0 --analytics 0 --append 0 --store 1 --cooccurrence 0 --setops 0 --canonicalize 0"
for v in base noxcd base noxcd; do
  L=$R/syzkaller_amd/libsyzgpu.so; [ $v != base ] && L=$R/syzkaller_amd/libsyzgpu_$v.so
  for cfg in "10000 50000" "100000 500000"; do
    set -- $cfg
    SYZGPU_LIB=$L timeout -k 10 300 python -u bench.py $LEGS --progs-per-gpu $1 --npcs $2 --steps 20 --warmup 3 > $OUT/b.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/b.log; exit $rc; }
    grep '^{' $OUT/b.log | tail -1 > $OUT/b.json
    python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$v', $1, d['ms_per_step'])" | tee -a $OUT/ab.log
  done
done
