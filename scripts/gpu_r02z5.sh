#!/bin/bash
# range guards on by default: full GPU suite (incl. the configs[1] full-shape test), A/B against
# the unguarded build at the bench shape
S=scripts/gpu_step.sh
B="--workload gossip --steps 10 --warmup 2 --no-cpu-baseline --no-vivaldi"
bash $S pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=8 && \
for i in 1 2; do
  RSF_LIB_PATH=$PWD/ab/lib_prev.so bash $S ab_prev$i 300 python3 bench.py $B && \
  bash $S ab_new$i 300 python3 bench.py $B || exit 1
done
