#!/bin/bash
# round 4 final tree (Vivaldi at 128-thread blocks): GPU suite, smoke, default bench line
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
bash $S pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread && \
bash $S smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" && \
bash $S bench_default 700 python -u bench.py
tail -2 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/smoke.log
