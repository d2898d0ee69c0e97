#!/bin/bash
# gpurun_retry.sh TIMEOUT OUTFILE CMD: one gpurun call, re-issued (after a pause) only when
# no box ran any part of the command (exit 3, or a transient verdict with no step run and
# no output).  A command that ran on a box -- even one whose box was then taken away -- is
# never repeated (a faulting command must not run twice).
lim=$1; out=$2; shift 2
# keep the previous call's outputs (outside the tree) before clearing
[ -n "$(ls -A gpurun_out 2>/dev/null)" ] && mkdir -p /tmp/gpurun_prev && cp -r gpurun_out /tmp/gpurun_prev/$(date +%s)
for a in $(seq 1 12); do
  rm -rf gpurun_out/*
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$@" > "$out" 2>&1
  rc=$?
  if [ $rc -eq 3 ]; then sleep 120; continue; fi
  if grep -q "status=transient" "$out" && python3 - <<'PY'
import json, sys
d = json.load(open("gpurun_out/.last_call.json"))
ran = bool(d.get("steps")) or bool((d.get("stdout_tail") or "").strip()) or (d.get("run_s") or 0) > 0
sys.exit(1 if ran else 0)
PY
  then sleep 120; continue; fi
  exit $rc
done
exit $rc
