#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool reports no box / a backoff (status=transient:
# nothing ran, nothing charged). A call that ran (ok or failed) is never repeated.
# Usage: bash tools/gpurun_when_free.sh OUTFILE TIMEOUT 'command'
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $OUT 2>&1
  if grep -q "status=transient\|already running\|slot(s) on this pod are busy" $OUT; then
    w=$(grep -o "retry in [0-9]*s" $OUT | grep -o "[0-9]*" | head -1); w=${w:-120}
    sleep $((w + 15)); continue
  fi
  break
done
echo "[when_free] done after $i submission(s)" >> $OUT
