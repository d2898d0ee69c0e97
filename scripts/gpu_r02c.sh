#!/bin/bash
S=scripts/gpu_step.sh
bash $S pytest_gossip 900 python -u -m pytest tests/test_gossip_gpu.py tests/test_dist_gpu.py tests/test_pushpull_gpu.py tests/test_reap_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread && \
bash $S r1 300 bash -c "cd experiments/libs/r1tree && python3 bench.py --workload gossip --steps 10 --warmup 2 --no-cpu-baseline" && \
bash $S cur 300 python3 bench.py --workload gossip --steps 10 --warmup 2 --no-cpu-baseline --no-vivaldi
