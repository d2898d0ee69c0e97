#!/bin/bash
# round 5: block-aggregated checker counts, tick before the ahead work; peers-ahead on/off in the regime; trace; default line
S=scripts/gpu_step.sh
bash $S pytest_deep 900 python -u -m pytest tests/test_deep_queue_gpu.py tests/test_gossip_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_deep.log && ! grep -q " failed\| error" gpurun_out/pytest_deep.log || exit 1
bash $S steady_inround 400 python -u experiments/steady_state.py 1000000 400 150 8704 10 inround || exit 1
RSF_PEERS_AHEAD=0 bash $S steady_inround_noahead 400 python -u experiments/steady_state.py 1000000 400 150 8704 10 inround || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash $S trace_inround 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_inr -o run -- python3 experiments/steady_state.py 1000000 360 150 8704 10 inround || exit 1
python3 experiments/trace_last.py gpurun_out/tr_inr/run_kernel_trace.csv 20 > gpurun_out/trace_inround_last20.txt 2>&1
bash $S bench_default 900 python -u bench.py
