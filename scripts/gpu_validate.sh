#!/bin/bash
# full validation: GPU tests, smoke, both default bench lines
S=scripts/gpu_step.sh
bash $S pytest_gpu 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread && \
bash $S smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" && \
bash $S bench_default 400 python -u bench.py && \
bash $S bench_vivaldi 400 python -u bench.py --workload vivaldi
