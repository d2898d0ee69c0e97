#!/bin/bash
# GPU tests + default gossip bench
S=scripts/gpu_step.sh
bash $S pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread && \
bash $S bench_default 400 python -u bench.py --no-cpu-baseline
