#!/bin/bash
# round 6: the deferred path without per-item decorations in LDS (small class 8 waves per CU,
# middle 4) -- the deep / gossip / regime parity tests, then a same-box A/B against the
# sector-aligned view build (abx/lib_aligned.so)
S=scripts/gpu_step.sh
bash $S pytest_deep 1100 python -u -m pytest tests/test_regime_gpu.py tests/test_deep_queue_gpu.py tests/test_gossip_gpu.py -v -s --timeout 1500 --timeout-method thread -x || exit 1
bash scripts/ab.sh abx 3 gossip aligned default || exit 1
grep -h "passed\|failed" gpurun_out/pytest_deep.log | tail -2
