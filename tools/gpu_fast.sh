#!/bin/bash
# Quick GPU iteration: the listed test files (default: all GPU tests), then the headline bench line
# without its side legs. Usage (repo root, through gpurun): bash tools/gpu_fast.sh TAG [test files...]
set -o pipefail
TAG=${1:-fast}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
T=${@:-tests}
timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python -u bench.py --novelty 0 --text 0 --hub 0 --analytics 0 --raw-steps 0 --cpu-baseline 0 \
  > $OUT/bench.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -20 $OUT/bench.log; exit $rc; }
python3 -c "
import json,sys
d=json.loads([l for l in open('$OUT/bench.log') if l.startswith('{')][-1])
print('ms_per_step', d['ms_per_step'], 'value', d['value'], 'roof', d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])
print(json.dumps(d['kernels_ms_per_step_serialized_pass']))
"
