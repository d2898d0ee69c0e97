#!/bin/bash
# the multi-GPU code path of the default line on one GPU: one RCCL rank (RSF_FORCE_SHARDED=1),
# gossip in the reference regime (ShardedGossip: bucket emission, in-round ticks per shard)
S=scripts/gpu_step.sh
RSF_FORCE_SHARDED=1 bash $S sharded_regime 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --steps 10 --no-extra-points --no-vivaldi --no-cpu-baseline
grep -h '^{' gpurun_out/sharded_regime.log | cut -c1-400
