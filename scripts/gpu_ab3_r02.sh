#!/bin/bash
S=scripts/gpu_step.sh
bash $S r1 300 bash -c "cd experiments/libs/r1tree && python3 bench.py --workload gossip --steps 10 --warmup 2 --no-cpu-baseline" && \
WLS=gossip bash $S ab 900 bash experiments/ab_variants.sh cur w6 w5 cur
