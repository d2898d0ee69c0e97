#!/bin/bash
# full GPU test suite + smoke + default gossip bench
S=scripts/gpu_step.sh
bash $S pytest_gpu 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread && \
bash $S smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" && \
bash $S bench_gossip 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline
