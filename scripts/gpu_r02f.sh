#!/bin/bash
S=scripts/gpu_step.sh
bash $S pytest_gossip 900 python -u -m pytest tests/test_gossip_gpu.py tests/test_dist_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread -k "two_shards or rccl or gloo or intent_rounds" && \
bash $S single 300 python3 bench.py --workload gossip --steps 10 --warmup 2 --no-cpu-baseline --no-vivaldi && \
RSF_FORCE_SHARDED=1 bash $S sharded1 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --workload gossip --steps 10 --warmup 2 --no-cpu-baseline --no-vivaldi
