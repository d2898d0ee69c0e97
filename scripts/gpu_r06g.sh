#!/bin/bash
# round 6: a fifth LDS class for the deferred path (kDeepLarge, queues up to ~5.7k items, 2 waves
# per CU) on top of the no-decoration LDS change -- the deep / gossip / regime parity tests, then
# a same-box A/B against the build without the large class (abx/lib_nodec.so)
S=scripts/gpu_step.sh
bash $S pytest_deep 900 python -u -m pytest tests/test_regime_gpu.py tests/test_deep_queue_gpu.py tests/test_gossip_gpu.py -v -s --timeout 800 --timeout-method thread -x || exit 1
grep -q " passed" gpurun_out/pytest_deep.log && ! grep -q "failed\|error" gpurun_out/pytest_deep.log || { grep -h "FAILED\|Error" gpurun_out/pytest_deep.log | head; exit 1; }
bash scripts/ab.sh abx 2 gossip nodec default || exit 1
grep -h "passed\|failed" gpurun_out/pytest_deep.log | tail -2
