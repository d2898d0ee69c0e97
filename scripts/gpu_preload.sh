#!/bin/bash
# code object loaded before the context's allocations: GPU suite, smoke, default bench, then the
# 1M-member bench (configs[1]) that faulted 3/3 before, and the opt-in configs[1] test
S=scripts/gpu_step.sh
bash $S pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread && \
bash $S smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" && \
bash $S bench_default 500 python -u bench.py && \
timeout -k 10 300 python -u bench.py --workload gossip --members 1000000 --steps 32 --warmup 3 --no-cpu-baseline --no-vivaldi > gpurun_out/bench_1m.log 2>&1
echo "bench_1m rc=$?"
tail -1 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/smoke.log; grep -h '^{' gpurun_out/bench_default.log gpurun_out/bench_1m.log | cut -c1-170; tail -1 gpurun_out/bench_1m.log | cut -c1-200
