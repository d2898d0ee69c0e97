#!/bin/bash
# The multi-GPU gossip code path (ShardedGossip over RCCL) on one GPU, beside the
# single-context bench in the same call: prices the exchange path's own overhead.
S=scripts/gpu_step.sh
bash $S bench_single 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline && \
RSF_FORCE_SHARDED=1 bash $S bench_sharded1 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline
