set -o pipefail
for e in "X=0" "SYZGPU_NW_DBG=1" "SYZGPU_NW_DBG=2"; do
  env $e timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --store 0 --text 0 --setops 0 --canonicalize 0 --hub 0 --analytics 0 --append 0 --cooccurrence 0 > gpurun_out/nwdbg_$e.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); n=d['novelty_config3']; print(sys.argv[2], n['ms_per_batch'], n['kernels_ms_per_batch'])" gpurun_out/nwdbg_$e.json $e
done
