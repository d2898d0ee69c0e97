#!/bin/bash
# round 4: non-temporal spill stores (nt) vs plain (base), configs[1] depth 4096, same box x2
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points --members 1000000"
for i in 1 2; do
  for v in nt base; do RSF_LIB_PATH=$PWD/ab/lib_$v.so bash $S deep_${v}_$i 300 $B --queue-depth 4096 || exit 1; done
done
for f in deep_nt_1 deep_base_1 deep_nt_2 deep_base_2; do grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phases_ms_per_round'].items()})"; done
