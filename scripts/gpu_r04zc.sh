#!/bin/bash
# round 4: final-tree Vivaldi profile (128-thread blocks) + a same-box 128 vs 256 block check
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
bash $S prof_viv 900 bash scripts/profile.sh r04d_viv vivaldi || exit 1
B="python3 -u bench.py --workload vivaldi --steps 10 --warmup 2 --no-cpu-baseline"
for v in v128 v256; do RSF_LIB_PATH=$PWD/ab/lib_$v.so bash $S ${v} 300 $B || exit 1; done
for f in v128 v256; do grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline',{}); print('$f', d['value'], round(d['ms_per_step'],3), r.get('avg_launch_ms'), r.get('frac'))"; done
