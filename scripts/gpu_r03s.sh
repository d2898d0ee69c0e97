#!/bin/bash
# Vivaldi round kernel at 64M: single LDS block + 4 waves/SIMD (spills), + late window loads, late window alone, vs default
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 -u bench.py --workload vivaldi --steps 10 --warmup 2 --no-cpu-baseline"
for i in 1 2; do
  bash $S def$i 200 $B && for v in v_lds1w4 v_latew4 v_late; do RSF_LIB_PATH=$PWD/ab/lib_$v.so bash $S ${v}_$i 200 $B || exit 1; done || exit 1
done
for f in def1 v_lds1w4_1 v_latew4_1 v_late_1 def2 v_lds1w4_2 v_latew4_2 v_late_2; do grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline',{}); print('$f', d['value'], round(d['ms_per_step'],3), r.get('avg_launch_ms'), r.get('frac'))"; done
