#!/bin/bash
# round 6: the small and middle deferred classes on the side stream beside the tiny class (joined
# before the full depth) -- the deep / regime / gossip / dist parity tests on that build
# (abx/lib_fork.so), then a same-box A/B against the tree
S=scripts/gpu_step.sh
RSF_LIB_PATH=$PWD/abx/lib_fork.so bash $S pytest_deep 900 python -u -m pytest tests/test_regime_gpu.py tests/test_deep_queue_gpu.py tests/test_gossip_gpu.py tests/test_dist_gpu.py -v -s --timeout 800 --timeout-method thread -x || exit 1
grep -q " passed" gpurun_out/pytest_deep.log && ! grep -q " failed\| error" gpurun_out/pytest_deep.log || { grep -h "FAILED\|Error" gpurun_out/pytest_deep.log | head; exit 1; }
bash scripts/ab.sh abx 3 gossip default fork || exit 1
grep -h "passed\|failed" gpurun_out/pytest_deep.log | tail -1
