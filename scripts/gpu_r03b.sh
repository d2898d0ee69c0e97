#!/bin/bash
# round 3: queue_cap > 64 after the LDS fences; the new GPU tests; then the whole suite
S=scripts/gpu_step.sh
bash $S q4_tests 400 python -u -m pytest tests/test_gossip_gpu.py -x -v --timeout 200 --timeout-method thread -k "queue_cap" && \
bash $S new_tests 500 python -u -m pytest tests/test_member_coalesce.py tests/test_dist_vivaldi_gpu.py tests/test_intern_gpu.py -x -v --timeout 300 --timeout-method thread -k "member or allgather or overflow or sharded" && \
bash $S pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -4 gpurun_out/q4_tests.log gpurun_out/new_tests.log; tail -3 gpurun_out/pytest_gpu.log
