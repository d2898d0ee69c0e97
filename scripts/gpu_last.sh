#!/bin/bash
# the exact final tree: smoke + default bench line (the driver's round-end bench)
S=scripts/gpu_step.sh
bash $S smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" && \
bash $S bench_default 500 python -u bench.py
tail -1 gpurun_out/smoke.log; grep -h '^{' gpurun_out/bench_default.log | cut -c1-160
