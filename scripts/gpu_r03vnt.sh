#!/bin/bash
# Vivaldi at 64M: non-temporal window-slot / index stores too (NT=3), no NT hints (NT=0), XCD block order, vs default
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 -u bench.py --workload vivaldi --steps 10 --warmup 2 --no-cpu-baseline"
for i in 1 2; do
  bash $S def$i 200 $B && for v in vnt3 vnt0 vxcd; do RSF_LIB_PATH=$PWD/ab/lib_$v.so bash $S ${v}_$i 200 $B || exit 1; done || exit 1
done
for f in def1 vnt3_1 vnt0_1 vxcd_1 def2 vnt3_2 vnt0_2 vxcd_2; do grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline',{}); print('$f', d['value'], r.get('avg_launch_ms'), r.get('frac'))"; done
