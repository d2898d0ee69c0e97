#!/bin/bash
# A/B timing of library variants built by build_variants.sh (gossip + vivaldi benches).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
for v in "$@"; do
  for w in ${WLS:-gossip vivaldi}; do
    RSF_LIB_PATH=$PWD/experiments/libs/lib_$v.so timeout -k 10 240 python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-vivaldi > gpurun_out/ab/${v}_$w.log 2>&1
    rc=$?
    echo "$v $w rc=$rc $(tail -1 gpurun_out/ab/${v}_$w.log | cut -c1-160)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
