S=scripts/gpu_step.sh
bash $S pytest_new 400 python -u -m pytest tests/test_reap_gpu.py tests/test_coalesce_gpu.py tests/test_gossip_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread && \
bash $S bench_gossip2m 600 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline
