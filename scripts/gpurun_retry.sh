#!/bin/bash
# gpurun_retry.sh TIMEOUT OUTFILE CMD: one gpurun call, re-issued (after a pause) only when
# gpurun reports that no box ran the command (exit 3 / a transient "retry" verdict); a
# command that ran on a box is never repeated.
lim=$1; out=$2; shift 2
for a in 1 2 3 4 5; do
  rm -rf gpurun_out/*
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$@" > "$out" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$out"; then sleep 60; continue; fi
  exit $rc
done
exit $rc
