#!/bin/bash
# round 4: deep emission specialised to the intent queue (mask template): deep tests,
# exact-key split diagnostics, q64 vs deep bench on one box, SQ counters of the deep point
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
bash $S deep_tests 900 python -u -m pytest tests/test_deep_queue_gpu.py -m gpu -v -x --timeout 600 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/deep_tests.log || exit 1
bash $S dprof30 300 env RSF_LIB_PATH=$PWD/ab/lib_dprof3.so python -u experiments/deep_prof.py 1000000 30 || exit 1
B="python -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points"
bash $S b1m_q64 300 $B --members 1000000 || exit 1
bash $S b1m_deep 300 $B --members 1000000 --queue-depth 4096 || exit 1

