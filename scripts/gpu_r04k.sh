#!/bin/bash
# round 4: deep path with cross-member prefetch: deep tests, diagnostics, q64 vs depth-4096
# bench on one box, SQ instruction counters of both (emit_kernel deep vs plain)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
bash $S deep_tests 900 python -u -m pytest tests/test_deep_queue_gpu.py -m gpu -v -x --timeout 600 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/deep_tests.log || exit 1
bash $S dprof30 300 env RSF_LIB_PATH=$PWD/ab/lib_dprof.so python -u experiments/deep_prof.py 1000000 30 || exit 1
B="python -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points"
bash $S b1m_q64 300 $B --members 1000000 || exit 1
bash $S b1m_deep 300 $B --members 1000000 --queue-depth 4096 || exit 1
bash $S pmc_q64 400 bash scripts/pmc_sq.sh q64 --workload gossip --no-vivaldi --no-extra-points --members 1000000 || exit 1
bash $S pmc_deep 400 bash scripts/pmc_sq.sh deep --workload gossip --no-vivaldi --no-extra-points --members 1000000 --queue-depth 4096
