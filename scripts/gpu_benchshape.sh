#!/bin/bash
# bench-shape bit-exact parity test (20k members, 4096 subjects, saturated queues)
S=scripts/gpu_step.sh
bash $S pytest_benchshape 400 python -u -m pytest tests/test_gossip_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "bench_shape" --durations=3
tail -8 gpurun_out/pytest_benchshape.log
