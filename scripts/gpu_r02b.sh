#!/bin/bash
# round 2: the new configs[3] / 64M Vivaldi / forget_node tests, then the churn bench leg
S=scripts/gpu_step.sh
bash $S pytest_new 900 python -u -m pytest tests/test_gossip_gpu.py tests/test_vivaldi_gpu.py -m gpu -v --timeout 600 --timeout-method thread -k "configs3 or forget or nan_defense or 64m or prune or ring" && \
bash $S bench_churn 600 python -u bench.py --workload churn --steps 20 --warmup 5
