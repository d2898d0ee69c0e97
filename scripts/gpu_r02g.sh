#!/bin/bash
# final tree: GPU suite, smoke, default bench line; then the 1M-member bench line (configs[1])
S=scripts/gpu_step.sh
bash $S pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread && \
bash $S smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" && \
bash $S bench_default 500 python -u bench.py && \
bash $S bench_1m 300 python -u bench.py --workload gossip --members 1000000 --steps 32 --warmup 3 --no-cpu-baseline --no-vivaldi
grep -h '^{' gpurun_out/bench_default.log gpurun_out/bench_1m.log | cut -c1-250; tail -2 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/bench_1m.log | cut -c1-300
