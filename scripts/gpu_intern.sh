#!/bin/bash
# device interning tests
S=scripts/gpu_step.sh
bash $S pytest_intern 300 python -u -m pytest tests/test_intern_gpu.py tests/test_codec_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread
cat gpurun_out/pytest_intern.log | tail -30
