#!/bin/bash
# Vivaldi round-kernel A/B: each library variant with 32-byte and 64-byte filter records.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
for v in "$@"; do
  for fr in ${FRS:-0 1}; do
    RSF_VIV_FR8=$fr RSF_LIB_PATH=$PWD/experiments/libs/lib_$v.so timeout -k 10 200 python3 bench.py --workload vivaldi --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab/viv_${v}_fr$fr.log 2>&1
    rc=$?
    echo "$v fr8=$fr rc=$rc $(tail -1 gpurun_out/ab/viv_${v}_fr$fr.log | cut -c60-140)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
