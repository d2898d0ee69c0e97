#!/bin/bash
# final tree without the profile passes: the whole GPU suite, smoke, the default bench line
S=scripts/gpu_step.sh
bash $S pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q " failed\| error" gpurun_out/pytest_gpu.log || exit 1
bash $S smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
bash $S bench_default 600 python -u bench.py
tail -2 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/smoke.log; grep -h '^{' gpurun_out/bench_default.log | cut -c1-200
