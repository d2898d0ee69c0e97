#!/bin/bash
# round 3: the 1M x 4096 shape after the hipCUB temporary-storage fix; canaries at 1M and 2M;
# then the whole GPU suite
S=scripts/gpu_step.sh
bash $S cfg1_test 600 python -u -m pytest tests/test_gossip_gpu.py -x -v --timeout 500 --timeout-method thread -k "configs1" && \
bash $S bench_1m 300 python -u bench.py --workload gossip --members 1000000 --no-vivaldi --no-cpu-baseline && \
bash $S bench_2m 300 python -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline && \
bash $S pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
grep -h '^{' gpurun_out/bench_1m.log gpurun_out/bench_2m.log | cut -c1-400; tail -3 gpurun_out/pytest_gpu.log
