#!/bin/bash
# A/B: pending entries loaded in emit's first round trip (32 lanes default; 0 = second round trip; 64)
S=scripts/gpu_step.sh
B="--workload gossip --steps 10 --warmup 2 --no-cpu-baseline --no-vivaldi"
bash $S pytest_gossip 600 python -u -m pytest tests/test_gossip_gpu.py tests/test_dist_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread && \
for i in 1 2; do
  for v in pe0 new pe64; do
    if [ $v = new ]; then bash $S ab_$v$i 300 python3 bench.py $B || exit 1
    else RSF_LIB_PATH=$PWD/ab/lib_$v.so bash $S ab_$v$i 300 python3 bench.py $B || exit 1; fi
  done
done
