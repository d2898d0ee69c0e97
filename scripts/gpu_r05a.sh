#!/bin/bash
# round 5: parity of the deep/gossip suites on the seal + peers-ahead build, then the
# steady-state run at depth 8192 and the peers-ahead A/B
S=scripts/gpu_step.sh
bash $S pytest_gossip 900 python -u -m pytest tests/test_deep_queue_gpu.py tests/test_gossip_gpu.py tests/test_reference_kats_gpu.py tests/test_dist_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_gossip.log && ! grep -q " failed\| error" gpurun_out/pytest_gossip.log || exit 1
bash $S steady8k 600 python -u experiments/steady_state.py 1000000 460 150 8192 10 || exit 1
timeout -k 10 600 bash scripts/ab_env.sh 2 "RSF_PEERS_AHEAD=0" "RSF_PEERS_AHEAD=1"
