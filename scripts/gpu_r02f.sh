#!/bin/bash
# round-2 closing measurements of the final tree: default bench line (both halves of the
# metric + CPU baselines), rocprofv3 kernel trace + FETCH/WRITE of the gossip round, forced
# multi-GPU code path on one GPU beside a single-context round
S=scripts/gpu_step.sh
bash $S pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread && \
bash $S smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" && \
bash $S bench_default 500 python -u bench.py && \
bash scripts/profile.sh r02f_gossip gossip --no-vivaldi && \
bash $S bench_single 300 python -u bench.py --workload gossip --steps 20 --warmup 3 --no-cpu-baseline --no-vivaldi && \
RSF_FORCE_SHARDED=1 bash $S bench_sharded1 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 1 --workload gossip --steps 20 --warmup 3 --no-cpu-baseline --no-vivaldi
