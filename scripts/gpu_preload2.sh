#!/bin/bash
# create() reads a code-object global before allocating: the 1M-member bench first, then the suite
S=scripts/gpu_step.sh
timeout -k 10 300 python -u bench.py --workload gossip --members 1000000 --steps 32 --warmup 3 --no-cpu-baseline --no-vivaldi > gpurun_out/bench_1m.log 2>&1
rc=$?; echo "bench_1m rc=$rc"; grep -h '^{' gpurun_out/bench_1m.log | cut -c1-170; tail -1 gpurun_out/bench_1m.log | cut -c1-200
[ $rc -ne 0 ] && exit 0
bash $S pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -1 gpurun_out/pytest_gpu.log
