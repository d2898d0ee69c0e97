#!/bin/bash
# round 4: Vivaldi 128-thread blocks with the XCD-contiguous block order vs without, same box x2
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 -u bench.py --workload vivaldi --steps 10 --warmup 2 --no-cpu-baseline"
for i in 1 2; do for v in v128 v128x; do RSF_LIB_PATH=$PWD/ab/lib_$v.so bash $S ${v}_$i 300 $B || exit 1; done; done
for i in 1 2; do for v in v128 v128x; do f=${v}_$i; grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline',{}); print('$f', d['value'], round(d['ms_per_step'],3), r.get('avg_launch_ms'), r.get('frac'))"; done; done
