#!/bin/bash
# gpu_ahead.sh: gossip parity suites, then the peers-ahead A/B at 2M (same box, alternating)
S=scripts/gpu_step.sh
bash $S pytest_gossip 900 python -u -m pytest tests/test_gossip_gpu.py tests/test_deep_queue_gpu.py tests/test_dist_gpu.py tests/test_reference_kats_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_gossip.log && ! grep -q "failed\|error" gpurun_out/pytest_gossip.log || exit 1
timeout -k 10 900 bash scripts/ab_env.sh 3 "RSF_PEERS_AHEAD=0" "RSF_PEERS_AHEAD=1"
