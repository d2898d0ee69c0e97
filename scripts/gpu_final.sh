#!/bin/bash
# final tree: GPU suite, smoke, default bench line (the driver's round-end commands)
S=scripts/gpu_step.sh
bash $S pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread && \
bash $S smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" && \
bash $S bench_default 500 python -u bench.py
tail -2 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/smoke.log; grep -h '^{' gpurun_out/bench_default.log | cut -c1-200
