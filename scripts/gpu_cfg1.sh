#!/bin/bash
# configs[1] full-shape property test + the gossip suite
S=scripts/gpu_step.sh
bash $S pytest_cfg1 600 python -u -m pytest tests/test_gossip_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread --durations=5
tail -15 gpurun_out/pytest_cfg1.log
