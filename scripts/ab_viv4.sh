#!/bin/bash
# Vivaldi round-kernel A/B of ab/lib_NAME.so variants (64M members, 10 timed rounds each), twice
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
for pass in 1 2; do
  for v in "$@"; do
    RSF_LIB_PATH=$PWD/ab/lib_$v.so timeout -k 10 200 python3 bench.py --workload vivaldi --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab/viv_${v}_p$pass.log 2>&1
    rc=$?
    python3 - "$v" "$pass" "gpurun_out/ab/viv_${v}_p$pass.log" <<'PY'
import json, sys
v, p, f = sys.argv[1:]
try:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(v, p, "ms/step %.3f" % d["ms_per_step"], "kernel_ms %.3f" % d["roofline"]["avg_launch_ms"], "frac %.3f" % d["roofline"]["frac"])
except Exception as e:
    print(v, p, "no result", e)
PY
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
