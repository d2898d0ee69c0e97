#!/bin/bash
# ab_env.sh ROUNDS "ENV_A" "ENV_B" ... : same-box A/B of environment settings on the default
# build (e.g. "RSF_PEERS_AHEAD=0" vs ""), alternating A B A B; bench args in $ABARGS.
rounds=$1; shift
mkdir -p gpurun_out/ab
for i in $(seq 1 "$rounds"); do
  k=0
  for e in "$@"; do
    k=$((k+1))
    env $e timeout -k 10 300 python3 -u bench.py --workload gossip --steps 20 --warmup 3 --no-cpu-baseline \
      --no-vivaldi --no-extra-points $ABARGS > "gpurun_out/ab/env${k}_$i.log" 2>&1
    rc=$?
    echo "[$e] #$i rc=$rc $(grep -h '^{' "gpurun_out/ab/env${k}_$i.log" | python3 -c '
import json, sys
for l in sys.stdin:
    d = json.loads(l); p = d.get("phases_ms_per_round") or {}
    print("ms/step %.3f" % d["ms_per_step"], " ".join("%s=%.3f" % (k.split()[0], v) for k, v in p.items()))')"
    case $rc in 0) ;; *) exit $rc ;; esac
  done
done
