#!/bin/bash
# full GPU test suite + smoke, one process each, fault-aware
S=scripts/gpu_step.sh
bash $S pytest_gpu 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread && \
bash $S smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
