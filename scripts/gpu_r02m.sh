#!/bin/bash
# pending lists of 128: GPU suite + alternating A/B against the round-start tree
S=scripts/gpu_step.sh
B="--workload gossip --steps 10 --warmup 2 --no-cpu-baseline --no-vivaldi"
bash $S pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread && \
for i in 1 2 3; do
  bash $S ab_base$i 300 bash -c "cd ab/base && python3 bench.py $B" && \
  bash $S ab_new$i 300 python3 bench.py $B || exit 1
done
