#!/bin/bash
# round 4: lean deferred path: deep tests (incl. intent-only prune pass-on), gossip suite, bench points
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
bash $S deep_tests 900 python -u -m pytest tests/test_deep_queue_gpu.py -m gpu -v -x --timeout 600 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/deep_tests.log || exit 1
B="python3 -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points --members 1000000"
bash $S b1m_q64 300 $B || exit 1
bash $S b1m_deep 300 $B --queue-depth 4096 || exit 1
bash $S kt_deep 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_deep -o kt -- python3 bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points --members 1000000 --steps 10 --queue-depth 4096
