#!/bin/bash
S=scripts/gpu_step.sh
bash $S pytest_viv 600 python -u -m pytest tests/test_dist_vivaldi_gpu.py tests/test_vivaldi_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread && \
RSF_DIST_BACKEND=gloo bash $S viv_gloo2 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --workload vivaldi --members 4000000 --members-total --steps 3 --warmup 1 --no-cpu-baseline && \
bash $S viv1 300 python3 bench.py --workload vivaldi --steps 10 --warmup 2 --no-cpu-baseline
