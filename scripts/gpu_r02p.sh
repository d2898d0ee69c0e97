#!/bin/bash
# A/B: cost of the merge's scattered view write-back (diagnostic variant, wrong results)
S=scripts/gpu_step.sh
B="--workload gossip --steps 10 --warmup 2 --no-cpu-baseline --no-vivaldi"
for i in 1 2; do
  bash $S ab_new$i 300 python3 bench.py $B && \
  RSF_LIB_PATH=$PWD/ab/lib_nostore.so bash $S ab_nostore$i 300 python3 bench.py $B || exit 1
done
