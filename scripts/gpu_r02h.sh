#!/bin/bash
S=scripts/gpu_step.sh
bash $S pytest_new 600 python -u -m pytest tests/test_snapshot_gpu.py tests/test_probe_gpu.py -m gpu -v --timeout 300 --timeout-method thread && \
bash $S pytest_all 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
