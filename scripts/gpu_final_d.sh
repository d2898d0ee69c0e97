#!/bin/bash
# round 6 final tree (after the bucket-key change): the whole GPU suite, smoke, the default bench line
S=scripts/gpu_step.sh
bash $S pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 800 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q " failed\| error" gpurun_out/pytest_gpu.log || { grep -h "FAILED\|Error" gpurun_out/pytest_gpu.log | head; exit 1; }
bash $S smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
bash $S bench_default 600 python -u bench.py || exit 1
tail -1 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/smoke.log; grep -h '^{' gpurun_out/bench_default.log | cut -c1-300
