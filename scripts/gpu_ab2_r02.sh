#!/bin/bash
# same-box: round-1 tree vs current tree (gossip), then the merge phase profile
S=scripts/gpu_step.sh
bash $S r1 300 bash -c "cd experiments/libs/r1tree && python3 bench.py --workload gossip --steps 10 --warmup 2 --no-cpu-baseline" && \
bash $S cur 300 python3 bench.py --workload gossip --steps 10 --warmup 2 --no-cpu-baseline --no-vivaldi && \
bash $S r1b 300 bash -c "cd experiments/libs/r1tree && python3 bench.py --workload gossip --steps 10 --warmup 2 --no-cpu-baseline" && \
bash $S curb 300 python3 bench.py --workload gossip --steps 10 --warmup 2 --no-cpu-baseline --no-vivaldi && \
RSF_LIB_PATH=$PWD/experiments/libs/lib_prof.so bash $S mprof 300 python3 experiments/merge_prof.py 2000000
