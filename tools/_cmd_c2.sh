set -o pipefail
OUT=gpurun_out/r06_c2b; mkdir -p $OUT; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in base noxcd mx0 px0 base noxcd mx0 px0 base noxcd mx0 px0; do
  L=$R/syzkaller_amd/libsyzgpu.so; [ $v != base ] && L=$R/syzkaller_amd/libsyzgpu_$v.so
  SYZGPU_LIB=$L timeout -k 10 300 python -u bench.py --progs-per-gpu 100000 --npcs 500000 --steps 20 --warmup 3 --cpu-baseline 0 --store 0 --text 0 --novelty 0 --hub 0 --analytics 0 --append 0 --cooccurrence 0 --setops 0 --canonicalize 0 --layout-change 0 > $OUT/b.json 2> $OUT/b.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/b.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$v', d['ms_per_step'])" | tee -a $OUT/ab.log
done
