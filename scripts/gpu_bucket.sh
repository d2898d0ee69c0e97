#!/bin/bash
# the bucket (multi-GPU) path's parity tests, then the forced one-rank line
S=scripts/gpu_step.sh
bash $S pytest_bucket 600 python -u -m pytest tests/test_dist_gpu.py tests/test_dist_vivaldi_gpu.py \
  "tests/test_deep_queue_gpu.py::test_deep_two_shards_buckets_equal_one_context" -m gpu -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_bucket.log && ! grep -q " failed\| error" gpurun_out/pytest_bucket.log || exit 1
bash scripts/gpu_sharded.sh
