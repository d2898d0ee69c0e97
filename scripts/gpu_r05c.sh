#!/bin/bash
# round 5: LDS-key QueueChecker prune + staggered ticks: deep suites, the steady state both ways, the default bench line
S=scripts/gpu_step.sh
bash $S pytest_deep 900 python -u -m pytest tests/test_deep_queue_gpu.py tests/test_gossip_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_deep.log && ! grep -q " failed\| error" gpurun_out/pytest_deep.log || exit 1
bash $S steady_sync 400 python -u experiments/steady_state.py 1000000 310 150 8704 10 || exit 1
bash $S steady_stag 400 python -u experiments/steady_state.py 1000000 520 150 8704 10 stagger || exit 1
bash $S bench_default 900 python -u bench.py
