#!/bin/bash
# ab.sh DIR ROUNDS WORKLOAD VARIANT... : same-box A/B of library builds DIR/lib_<VARIANT>.so
# (loaded through RSF_LIB_PATH; "default" = the in-tree build), each variant timed ROUNDS
# times in alternating order (A B A B ...), so clock drift on the box shows up in every
# variant alike.  Extra bench args in $ABARGS.  Logs: gpurun_out/ab/<variant>_<i>.log;
# one summary line per run.
dir=$1; rounds=$2; wl=$3; shift 3
mkdir -p gpurun_out/ab
for i in $(seq 1 "$rounds"); do
  for v in "$@"; do
    lib=""
    [ "$v" != default ] && lib="RSF_LIB_PATH=$PWD/$dir/lib_$v.so"
    env $lib timeout -k 10 300 python3 -u bench.py --workload "$wl" --steps 20 --warmup 3 --no-cpu-baseline \
      --no-vivaldi --no-extra-points $ABARGS > "gpurun_out/ab/${v}_$i.log" 2>&1
    rc=$?
    echo "$v #$i rc=$rc $(grep -h '^{' "gpurun_out/ab/${v}_$i.log" | python3 -c '
import json, sys
for l in sys.stdin:
    d = json.loads(l); p = d.get("phases_ms_per_round") or {}
    print("ms/step %.3f" % d["ms_per_step"], " ".join("%s=%.3f" % (k.split()[0], v) for k, v in p.items()),
          "kernel %.3f" % d["roofline"]["avg_launch_ms"])')"
    case $rc in 0) ;; *) exit $rc ;; esac
  done
done
