#!/bin/bash
# A/B: merge receivers per wave and register cap after the queue left the merge
S=scripts/gpu_step.sh
B="--workload gossip --steps 10 --warmup 2 --no-cpu-baseline --no-vivaldi"
for i in 1 2; do
  bash $S ab_new$i 300 python3 bench.py $B && \
  for v in w8 p4 p16 p4w8; do RSF_LIB_PATH=$PWD/ab/lib_$v.so bash $S ab_$v$i 300 python3 bench.py $B || exit 1; done
done
