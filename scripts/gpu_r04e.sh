#!/bin/bash
# round 4: the one-wave deferred-emission path: deep tests, then configs[1] q64 vs depth 4096
S=scripts/gpu_step.sh
bash $S deep_tests 900 python -u -m pytest tests/test_deep_queue_gpu.py -m gpu -v -x --timeout 600 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/deep_tests.log || exit 1
B="python -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points"
bash $S b1m_q64 300 $B --members 1000000 || exit 1
bash $S b1m_deep 300 $B --members 1000000 --queue-depth 4096 || exit 1
bash $S b1m_deep_s30 300 $B --members 1000000 --queue-depth 4096 --settle 30
