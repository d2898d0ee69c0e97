#!/bin/bash
# emission: queue_cap-64 specialisation (FULL) + one lane-distributed bookkeeping store (cur),
# FULL without the combined store (nostore1), HEAD; parity of cur
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points"
bash $S tests 500 python -u -m pytest tests/test_gossip_gpu.py tests/test_dist_gpu.py tests/test_snapshot_gpu.py tests/test_pushpull_gpu.py tests/test_reap_gpu.py -x -q --timeout 200 --timeout-method thread && \
for i in 1 2; do
  RSF_LIB_PATH=$PWD/ab/lib_head.so bash $S head$i 200 $B && bash $S cur$i 200 $B && RSF_LIB_PATH=$PWD/ab/lib_nostore1.so bash $S nostore1_$i 200 $B || exit 1
done
tail -2 gpurun_out/tests.log
for f in head1 cur1 nostore1_1 head2 cur2 nostore1_2; do grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phases_ms_per_round'].items()})"; done
