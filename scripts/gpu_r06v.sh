#!/bin/bash
# round 6: with 4 items per lane the smallest deferred class needs 165 VGPRs (three waves per
# SIMD), so its 15 KB of LDS set its occupancy (10 waves per CU); the deferred path's histogram,
# head-gather and re-rank scratch aliased in LDS (13.4 KB: 12 waves per CU) -- the deep / regime /
# gossip / dist parity tests, then a same-box A/B against HEAD (abx/lib_prev.so)
S=scripts/gpu_step.sh
bash $S pytest_deep 900 python -u -m pytest tests/test_regime_gpu.py tests/test_deep_queue_gpu.py tests/test_gossip_gpu.py tests/test_dist_gpu.py -v -s --timeout 800 --timeout-method thread -x || exit 1
grep -q " passed" gpurun_out/pytest_deep.log && ! grep -q " failed\| error" gpurun_out/pytest_deep.log || { grep -h "FAILED\|Error" gpurun_out/pytest_deep.log | head; exit 1; }
bash scripts/ab.sh abx 3 gossip prev default || exit 1
grep -h "passed\|failed" gpurun_out/pytest_deep.log | tail -1
