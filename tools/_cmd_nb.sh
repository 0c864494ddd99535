set -o pipefail
OUT=gpurun_out/r06_nb; mkdir -p $OUT; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for V in base b15 hs512 hs2048; do
  E=""; L=$R/syzkaller_amd/libsyzgpu_dev.so
  [ $V = base ] && L=$R/syzkaller_amd/libsyzgpu.so
  [ $V = b15 ] && E="SYZGPU_NW_BITS=15"
  [ $V = hs512 ] && E="SYZGPU_NW_HSPARSE=512"
  [ $V = hs2048 ] && E="SYZGPU_NW_HSPARSE=2048"
  env SYZGPU_LIB=$L $E timeout -k 10 300 python3 -u tools/nov_bench.py 4 > $OUT/nov_$V.log 2>&1 || { tail -5 $OUT/nov_$V.log; exit 1; }
  echo "== $V"; python3 -c "
import json,sys
t=open('$OUT/nov_$V.log').read(); j=json.loads(t[t.index('{'):])
print(j['ms_per_batch'], j['kernels_ms_per_batch'], 'wide', j['wide_span']['ms_per_batch'])"
done
