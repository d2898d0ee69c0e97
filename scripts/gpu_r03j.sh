#!/bin/bash
# emission queue-major (q_pick_peers, the default) vs per-peer lazy picks; + first 32 pending
# entries speculatively in round trip 1; parity of the default; phase split of the default
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points"
bash $S multi_tests 500 python -u -m pytest tests/test_gossip_gpu.py tests/test_dist_gpu.py tests/test_snapshot_gpu.py tests/test_pushpull_gpu.py -x -q --timeout 200 --timeout-method thread && \
for i in 1 2; do
  RSF_LIB_PATH=$PWD/ab/lib_lazy.so bash $S lazy$i 200 $B && bash $S multi$i 200 $B && RSF_LIB_PATH=$PWD/ab/lib_spec32.so bash $S spec32_$i 200 $B || exit 1
done
RSF_LIB_PATH=$PWD/ab/lib_eprof.so bash $S emit_prof 300 python3 experiments/merge_prof.py 2000000 emit
tail -2 gpurun_out/multi_tests.log
for f in lazy1 multi1 spec32_1 lazy2 multi2 spec32_2; do grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phases_ms_per_round'].items()})"; done
grep '{' gpurun_out/emit_prof.log
