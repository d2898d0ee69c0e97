#!/bin/bash
# round 4: deep-queue tests incl. the long-queue capacity-class test
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
bash $S deep_tests 900 python -u -m pytest tests/test_deep_queue_gpu.py -m gpu -v -x --timeout 600 --timeout-method thread
