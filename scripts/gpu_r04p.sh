#!/bin/bash
# round 4: sorted tail prefix (deep path writes it, emission merges it): deep tests, gossip
# tests, diagnostics, q64 vs deep bench on one box, kernel trace of the deep point
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
bash $S deep_tests 900 python -u -m pytest tests/test_deep_queue_gpu.py -m gpu -v -x --timeout 600 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/deep_tests.log || exit 1
bash $S dprof30 300 env RSF_LIB_PATH=$PWD/ab/lib_dprof4.so python -u experiments/deep_prof.py 1000000 30 || exit 1
B="python3 -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points --members 1000000"
bash $S b1m_q64 300 $B || exit 1
bash $S b1m_deep 300 $B --queue-depth 4096 || exit 1
bash $S kt_deep 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_deep -o kt -- python3 bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points --members 1000000 --steps 10 --queue-depth 4096
