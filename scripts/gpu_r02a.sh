#!/bin/bash
# round 2: full GPU suite, then the default driver bench (gossip + Vivaldi legs, CPU baselines)
S=scripts/gpu_step.sh
bash $S pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread && \
bash $S bench_default 600 python -u bench.py --gpus 1 --steps 20 --warmup 5
