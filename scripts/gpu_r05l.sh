#!/bin/bash
# round 5: checker unroll A/B (full tick at 1M x 7.1k items), smoke, default bench line
S=scripts/gpu_step.sh
for v in default u32 u16x16 default; do
  lib=""; [ "$v" != default ] && lib="RSF_LIB_PATH=$PWD/abx/lib_$v.so"
  env $lib bash $S chk_$v 300 python -u experiments/check_prof.py 1000000 300 || exit 1
done
bash $S smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
bash $S bench_default 900 python -u bench.py
grep -h '^{' gpurun_out/chk_*.log
