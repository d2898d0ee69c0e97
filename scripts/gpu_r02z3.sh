#!/bin/bash
# pending lists as one array of 12-B entries: GPU suite + same-box A/B against the SoA lists
S=scripts/gpu_step.sh
B="--workload gossip --steps 10 --warmup 2 --no-cpu-baseline --no-vivaldi"
bash $S pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread && \
for i in 1 2 3; do
  RSF_LIB_PATH=$PWD/ab/lib_prev.so bash $S ab_prev$i 300 python3 bench.py $B && \
  bash $S ab_new$i 300 python3 bench.py $B || exit 1
done
