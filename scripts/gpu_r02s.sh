#!/bin/bash
# A/B: several senders per emit wave (next sender's first round trip prefetched)
S=scripts/gpu_step.sh
B="--workload gossip --steps 10 --warmup 2 --no-cpu-baseline --no-vivaldi"
for i in 1 2; do
  bash $S ab_new$i 300 python3 bench.py $B && \
  for v in epw2 epw4; do RSF_LIB_PATH=$PWD/ab/lib_$v.so bash $S ab_$v$i 300 python3 bench.py $B || exit 1; done
done
