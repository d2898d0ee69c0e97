#!/bin/bash
S=scripts/gpu_step.sh
RSF_PRUNE_FRAC=0 bash $S p0 300 python3 bench.py --workload gossip --steps 10 --warmup 2 --no-cpu-baseline --no-vivaldi && \
bash $S p1 300 python3 bench.py --workload gossip --steps 10 --warmup 2 --no-cpu-baseline --no-vivaldi && \
bash $S r1 300 bash -c "cd experiments/libs/r1tree && python3 bench.py --workload gossip --steps 10 --warmup 2 --no-cpu-baseline"
