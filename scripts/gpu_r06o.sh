#!/bin/bash
# round 6: the small deferred class also with one 256-thread block per member (recent mode kept; four waves share
# the tail load, the key range, the selects, the gather and the tail store) -- the deep / gossip
# / regime / bucket parity tests, then a same-box A/B against the one-wave class
# (abx/lib_smallwave.so) and against the tiny class in blocks too (abx/lib_tinyblock.so)
S=scripts/gpu_step.sh
bash $S pytest_deep 900 python -u -m pytest tests/test_regime_gpu.py tests/test_deep_queue_gpu.py tests/test_gossip_gpu.py tests/test_dist_gpu.py -v -s --timeout 800 --timeout-method thread -x || exit 1
grep -q " passed" gpurun_out/pytest_deep.log && ! grep -q " failed\| error" gpurun_out/pytest_deep.log || { grep -h "FAILED\|Error" gpurun_out/pytest_deep.log | head; exit 1; }
bash scripts/ab.sh abx 2 gossip smallwave default tinyblock || exit 1
grep -h "passed\|failed" gpurun_out/pytest_deep.log | tail -1
