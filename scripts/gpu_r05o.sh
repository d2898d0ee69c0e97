#!/bin/bash
# round 5: one full-depth launch for lists 1 and 4; parity + same-box A/B against two launches
S=scripts/gpu_step.sh
bash $S pytest_deep 900 python -u -m pytest tests/test_deep_queue_gpu.py tests/test_gossip_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_deep.log && ! grep -q " failed\| error" gpurun_out/pytest_deep.log || exit 1
for v in default twolaunch default twolaunch; do
  lib=""; [ "$v" != default ] && lib="RSF_LIB_PATH=$PWD/abx/lib_$v.so"
  env $lib bash $S ss_$v 300 python -u experiments/steady_state.py 1000000 380 150 8704 10 inround || exit 1
  grep '"round": 3[5-8]0' gpurun_out/ss_$v.log | cut -c1-60 >> gpurun_out/ab_launch.txt
  echo "-- $v" >> gpurun_out/ab_launch.txt
done
