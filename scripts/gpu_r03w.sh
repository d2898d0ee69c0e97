#!/bin/bash
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
bash $S tests 400 python -u -m pytest tests/test_gossip_gpu.py -x -v --timeout 200 --timeout-method thread -k "emission_pick_paths"
tail -8 gpurun_out/tests.log
