#!/bin/bash
S=scripts/gpu_step.sh
bash $S pytest_snap 600 python -u -m pytest tests/test_snapshot_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread && \
bash $S pytest_all 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
