#!/bin/bash
# round 4: merge-class kernels at 4 (default) / 2 / 1 waves per block, 2M gossip round, same box x2
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points"
for i in 1 2; do
  for v in w4 w2 w1; do RSF_LIB_PATH=$PWD/ab/lib_$v.so bash $S ${v}_$i 300 $B || exit 1; done
done
for i in 1 2; do for v in w4 w2 w1; do f=${v}_$i; grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value']/1e8,3), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phases_ms_per_round'].items()})"; done; done
