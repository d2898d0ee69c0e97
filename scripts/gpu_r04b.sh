#!/bin/bash
# round 4: deep-queue tests, then the other new tests, then the whole GPU suite
S=scripts/gpu_step.sh
bash $S deep_tests 900 python -u -m pytest tests/test_deep_queue_gpu.py -m gpu -v -x --timeout 600 --timeout-method thread || exit 1
bash $S new_tests 600 python -u -m pytest tests/test_reference_kats_gpu.py "tests/test_gossip_gpu.py::test_bench_shape_bit_exact" tests/test_coalesce_gpu.py tests/test_member_coalesce.py tests/test_swim_gpu.py "tests/test_dist_gpu.py::test_configs2_shard_rccl_equal_one_context" -m gpu -v --timeout 500 --timeout-method thread || exit 1
bash $S pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
