#!/bin/bash
# round 3: the 1M x 4096 shape after the hipCUB temporary-storage fix; the GPU suite
# (lazy re-rank emission, queue_cap up to 256, member-event log + coalescer); benches at 1M
# and 2M with canaries; emission A/B without the deferred re-rank; a 256-slot point
S=scripts/gpu_step.sh
bash $S cfg1_test 600 python -u -m pytest tests/test_gossip_gpu.py -x -v --timeout 500 --timeout-method thread -k "configs1" && \
bash $S pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread && \
bash $S bench_1m 300 python -u bench.py --workload gossip --members 1000000 --no-vivaldi --no-cpu-baseline && \
bash $S bench_2m 300 python -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline && \
RSF_LIB_PATH=$PWD/ab/lib_nolazy.so bash $S bench_2m_nolazy 300 python -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline && \
bash $S bench_1m_q256 300 python -u bench.py --workload gossip --members 1000000 --queue-cap 256 --settle 3 --warmup 1 --steps 6 --no-vivaldi --no-cpu-baseline
grep -h '^{' gpurun_out/bench_*.log | cut -c1-300; tail -3 gpurun_out/pytest_gpu.log
