#!/bin/bash
# round 5: same-box A/B of the sealed pulls in the reference regime (steady state, 1M)
S=scripts/gpu_step.sh
for v in default nopull default nopull; do
  lib=""; [ "$v" != default ] && lib="RSF_LIB_PATH=$PWD/abx/lib_$v.so"
  env $lib bash $S ss_$v 300 python -u experiments/steady_state.py 1000000 380 150 8704 10 inround || exit 1
  grep '"round": 3[5-8]0' gpurun_out/ss_$v.log | cut -c1-60 >> gpurun_out/ab_pull.txt
  echo "-- $v" >> gpurun_out/ab_pull.txt
done
