S=scripts/gpu_step.sh
bash $S pytest_pp 400 python -u -m pytest tests/test_pushpull_gpu.py tests/test_gossip_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread && \
bash $S bench_pp 500 python -u bench.py --workload pushpull --steps 3 --warmup 1
