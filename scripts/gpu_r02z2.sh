#!/bin/bash
# pending-append layouts in the merge's access pattern; bucket exchange without decorations:
# multi-GPU parity tests, forced one-rank RCCL round and single-context round
S=scripts/gpu_step.sh
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -w -o gpurun_out/view_floor experiments/view_floor.hip && \
bash $S view_floor 120 gpurun_out/view_floor && cat gpurun_out/view_floor.log && \
bash $S pytest_dist 400 python -u -m pytest tests/test_dist_gpu.py tests/test_gossip_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread && \
bash $S bench_single 300 python -u bench.py --workload gossip --steps 20 --warmup 3 --no-cpu-baseline --no-vivaldi && \
RSF_FORCE_SHARDED=1 bash $S bench_sharded1 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 1 --workload gossip --steps 20 --warmup 3 --no-cpu-baseline --no-vivaldi
