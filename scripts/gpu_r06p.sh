#!/bin/bash
# round 6: the checker lists its deep queues at fixed places (no global atomic per listed
# queue) and check_stream_kernel reads its next entry ahead -- the deep / gossip / regime /
# bucket parity tests (with the long-queue cases that prune inside the block classes), then a
# same-box A/B against HEAD (abx/lib_prev.so) and against this tree plus the smallest class at
# 12 waves per CU (abx/lib_tiny12.so: the LDS scratch aliased, three waves per SIMD)
S=scripts/gpu_step.sh
bash $S pytest_deep 900 python -u -m pytest tests/test_regime_gpu.py tests/test_deep_queue_gpu.py tests/test_gossip_gpu.py tests/test_dist_gpu.py -v -s --timeout 800 --timeout-method thread -x || exit 1
grep -q " passed" gpurun_out/pytest_deep.log && ! grep -q " failed\| error" gpurun_out/pytest_deep.log || { grep -h "FAILED\|Error" gpurun_out/pytest_deep.log | head; exit 1; }
bash scripts/ab.sh abx 2 gossip prev default tiny12 || exit 1
grep -h "passed\|failed" gpurun_out/pytest_deep.log | tail -1
