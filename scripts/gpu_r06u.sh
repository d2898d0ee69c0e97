#!/bin/bash
# round 6: the deferred path's items in flight per lane (RSF_DEEP_U) at 4 instead of 8 -- the deep
# / regime / gossip / dist parity tests on that build (abx/lib_du4.so), then a same-box A/B of
# 8 (the tree), 4, 2 and 6
S=scripts/gpu_step.sh
RSF_LIB_PATH=$PWD/abx/lib_du4.so bash $S pytest_deep 900 python -u -m pytest tests/test_regime_gpu.py tests/test_deep_queue_gpu.py tests/test_gossip_gpu.py tests/test_dist_gpu.py -v -s --timeout 800 --timeout-method thread -x || exit 1
grep -q " passed" gpurun_out/pytest_deep.log && ! grep -q " failed\| error" gpurun_out/pytest_deep.log || { grep -h "FAILED\|Error" gpurun_out/pytest_deep.log | head; exit 1; }
bash scripts/ab.sh abx 3 gossip default du4 du2 du6 || exit 1
grep -h "passed\|failed" gpurun_out/pytest_deep.log | tail -1
