#!/bin/bash
# round 6: the bench-regime bit-exact test, then the rest of the GPU suite
S=scripts/gpu_step.sh
bash $S regime_test 1000 python -u -m pytest tests/test_regime_gpu.py -x -v -s --timeout 1500 --timeout-method thread || exit 1
bash $S pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --deselect tests/test_regime_gpu.py::test_bench_regime_bit_exact || exit 1
grep -h "passed\|failed" gpurun_out/regime_test.log gpurun_out/pytest_gpu.log | tail -3
