#!/bin/bash
# deferred re-queues v2 (queue-held decorations, origination headroom): GPU suite + A/B
S=scripts/gpu_step.sh
B="--workload gossip --steps 10 --warmup 2 --no-cpu-baseline --no-vivaldi"
bash $S pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread && \
bash $S ab_base 300 bash -c "cd ab/base && python3 bench.py $B" && \
bash $S ab_new 300 python3 bench.py $B && \
RSF_LIB_PATH=$PWD/ab/lib_rt1.so bash $S ab_rt1 300 python3 bench.py $B && \
RSF_LIB_PATH=$PWD/ab/lib_w8.so bash $S ab_w8 300 python3 bench.py $B && \
bash $S ab_new2 300 python3 bench.py $B && \
RSF_LIB_PATH=$PWD/ab/lib_rt1.so bash $S ab_rt12 300 python3 bench.py $B
