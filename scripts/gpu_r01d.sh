#!/bin/bash
# Round-1 refresh after the merge-kernel changes: GPU tests, smoke, gossip rocprofv3 trace +
# FETCH/WRITE passes, default bench line, and a 2-rank host-staged (gloo) rehearsal of the
# Vivaldi multi-GPU bench with the table refreshed every 8 rounds.
S=scripts/gpu_step.sh
bash $S pytest_gpu 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread && \
bash $S smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" && \
bash $S prof_gossip 600 bash scripts/profile.sh gossip_r01d gossip && \
bash $S bench_default 400 python -u bench.py && \
RSF_DIST_BACKEND=gloo bash $S viv_gloo_r8 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --workload vivaldi --members 2000000 \
  --refresh-every 8 --steps 16 --warmup 2 --no-cpu-baseline
