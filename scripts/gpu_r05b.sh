#!/bin/bash
# round 5: deep suites on the reserve + in-place-fallback build, then the steady-state run at depth 8704
S=scripts/gpu_step.sh
bash $S pytest_deep 900 python -u -m pytest tests/test_deep_queue_gpu.py tests/test_gossip_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_deep.log && ! grep -q " failed\| error" gpurun_out/pytest_deep.log || exit 1
bash $S steady8k 600 python -u experiments/steady_state.py 1000000 460 150 8704 10
