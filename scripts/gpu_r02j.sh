#!/bin/bash
# deferred re-queues: GPU suite, then same-box A/B of the gossip round (base tree vs new vs new+8 waves)
S=scripts/gpu_step.sh
B="--workload gossip --steps 10 --warmup 2 --no-cpu-baseline --no-vivaldi"
bash $S pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread && \
bash $S ab_base 300 bash -c "cd ab/base && python3 bench.py $B" && \
bash $S ab_new 300 python3 bench.py $B && \
RSF_LIB_PATH=$PWD/ab/lib_w8.so bash $S ab_w8 300 python3 bench.py $B && \
bash $S ab_base2 300 bash -c "cd ab/base && python3 bench.py $B" && \
bash $S ab_new2 300 python3 bench.py $B
