#!/bin/bash
# round 6: the Vivaldi pipe kernel at 192 threads per block (RSF_VIV_BLOCK) -- the Vivaldi GPU
# tests on that build (abx/lib_vb192.so), then a same-box A/B against 128 (the tree), 3 rounds
S=scripts/gpu_step.sh
RSF_LIB_PATH=$PWD/abx/lib_vb192.so bash $S pytest_viv 600 python -u -m pytest tests/test_vivaldi_gpu.py tests/test_dist_vivaldi_gpu.py -v --timeout 500 --timeout-method thread -x || exit 1
grep -q " passed" gpurun_out/pytest_viv.log && ! grep -q " failed\| error" gpurun_out/pytest_viv.log || { grep -h "FAILED\|Error" gpurun_out/pytest_viv.log | head; exit 1; }
bash scripts/ab.sh abx 3 vivaldi default vb192 || exit 1
grep -h "passed\|failed" gpurun_out/pytest_viv.log | tail -1
