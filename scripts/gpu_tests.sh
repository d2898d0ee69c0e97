#!/bin/bash
# GPU test suite only (optionally a subset: scripts/gpu_tests.sh tests/test_x.py ...)
S=scripts/gpu_step.sh
T=${@:-tests}
bash $S pytest_gpu 900 python -u -m pytest $T -m gpu -v --timeout 300 --timeout-method thread
