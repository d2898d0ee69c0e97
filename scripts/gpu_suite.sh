#!/bin/bash
# the whole GPU suite (the driver's round-end pytest), log to gpurun_out/pytest_gpu.log
S=scripts/gpu_step.sh
bash $S pytest_gpu 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
tail -3 gpurun_out/pytest_gpu.log
