#!/bin/bash
# round 4: configs[1] at 64-slot queues vs 4096-deep intent queues (same call), then the 2M headline
S=scripts/gpu_step.sh
B="python -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points"
bash $S b1m_q64 300 $B --members 1000000 || exit 1
bash $S b1m_deep 300 $B --members 1000000 --queue-depth 4096 || exit 1
bash $S b1m_deep_s30 300 $B --members 1000000 --queue-depth 4096 --settle 30 || exit 1
bash $S b2m_q64 300 $B
