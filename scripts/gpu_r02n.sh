#!/bin/bash
# thread-per-receiver merge: GPU suite + A/B (wave merge, register caps)
S=scripts/gpu_step.sh
B="--workload gossip --steps 10 --warmup 2 --no-cpu-baseline --no-vivaldi"
bash $S pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread && \
for i in 1 2; do
  bash $S ab_new$i 300 python3 bench.py $B && \
  RSF_LIB_PATH=$PWD/ab/lib_wave.so bash $S ab_wave$i 300 python3 bench.py $B && \
  RSF_LIB_PATH=$PWD/ab/lib_lb8.so bash $S ab_lb8$i 300 python3 bench.py $B && \
  RSF_LIB_PATH=$PWD/ab/lib_lb6.so bash $S ab_lb6$i 300 python3 bench.py $B || exit 1
done
