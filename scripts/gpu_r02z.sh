#!/bin/bash
# re-entry check of the current tree: GPU suite, smoke, default bench line, rocprofv3 of the gossip round
S=scripts/gpu_step.sh
bash $S pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread && \
bash $S smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" && \
bash $S bench_default 500 python -u bench.py && \
bash scripts/profile.sh r02z_gossip gossip --no-vivaldi
