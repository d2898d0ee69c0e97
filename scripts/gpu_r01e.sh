#!/bin/bash
# Round-1 closing refresh (tag r01f): GPU tests, smoke, gossip rocprofv3 trace + FETCH/WRITE passes,
# both default bench lines (with CPU baselines), and the forced one-rank multi-GPU path.
S=scripts/gpu_step.sh
bash $S pytest_gpu 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread && \
bash $S smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" && \
bash $S prof_gossip 600 bash scripts/profile.sh gossip_r01f gossip && \
bash $S bench_default 400 python -u bench.py && \
bash $S bench_vivaldi 400 python -u bench.py --workload vivaldi && \
bash scripts/gpu_sharded1.sh
