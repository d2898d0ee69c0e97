#!/bin/bash
# round 3: the new / changed GPU tests, the whole suite, then the emission A/B and profiles
S=scripts/gpu_step.sh
bash $S q4_tests 400 python -u -m pytest tests/test_gossip_gpu.py -v --timeout 200 --timeout-method thread -k "queue_cap" && \
bash $S new_tests 500 python -u -m pytest tests/test_member_coalesce.py tests/test_dist_vivaldi_gpu.py tests/test_intern_gpu.py tests/test_vivaldi_gpu.py -v --timeout 300 --timeout-method thread -k "member or allgather or overflow or sharded or c1" && \
bash $S pytest_gpu 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread && \
bash scripts/gpu_r03c.sh
grep -E "PASS|FAIL" gpurun_out/q4_tests.log gpurun_out/new_tests.log | cut -c1-150; tail -3 gpurun_out/pytest_gpu.log
