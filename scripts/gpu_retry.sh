#!/bin/bash
# gpu_retry.sh OUTFILE CMD : retries gpurun only while it reports a transient
# infrastructure failure (no box / box not responding), never after the command ran.
out=$1; shift
for i in 1 2 3 4 5 6; do
  timeout 1500 /usr/local/graft/bin/gpurun --timeout 900 -- "$1" > "$out" 2>&1
  if grep -q "status=transient\|rc=3\|backing off" "$out" && ! grep -q "status=ok\|status=fail" "$out"; then
    sleep 45; continue
  fi
  break
done
