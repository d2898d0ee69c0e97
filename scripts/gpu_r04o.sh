#!/bin/bash
# round 4: where the deep emission's extra time goes (timing diagnostics; results differ):
# no tail writes on spill, no pick checks against the tails; the default build beside them
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points --members 1000000"
for v in dbase dnsw dnck; do
  RSF_LIB_PATH=$PWD/ab/lib_$v.so bash $S deep_$v 300 $B --queue-depth 4096 || exit 1
done
RSF_LIB_PATH=$PWD/ab/lib_dbase.so bash $S q64_dbase 300 $B || exit 1
for f in deep_dbase deep_dnsw deep_dnck q64_dbase; do grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phases_ms_per_round'].items()}, d.get('deep_path_members_per_round'))"; done
