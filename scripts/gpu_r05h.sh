#!/bin/bash
# round 5: checker prune with one select and no refill; sequential deep classes and in-round tick
S=scripts/gpu_step.sh
bash $S pytest_deep 900 python -u -m pytest tests/test_deep_queue_gpu.py tests/test_gossip_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_deep.log && ! grep -q " failed\| error" gpurun_out/pytest_deep.log || exit 1
bash $S check_prof 300 python -u experiments/check_prof.py 1000000 300 || exit 1
bash $S steady_inround 400 python -u experiments/steady_state.py 1000000 400 150 8704 10 inround || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash $S trace_inround 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_inr -o run -- python3 experiments/steady_state.py 1000000 360 150 8704 10 inround || exit 1
python3 experiments/trace_last.py gpurun_out/tr_inr/run_kernel_trace.csv 20 > gpurun_out/trace_inround_last20.txt 2>&1
