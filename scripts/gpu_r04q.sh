#!/bin/bash
# round 4: emission split into emit_kernel / emit_kernel_deep: full GPU suite, then the deep
# emission with an SGPR cap (occupancy 8, 11 SGPRs spilled to lanes) against the default, x2
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
bash $S pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_gpu.log || exit 1
B="python3 -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points --members 1000000"
for i in 1 2; do
  for v in dbase s94; do RSF_LIB_PATH=$PWD/ab/lib_$v.so bash $S deep_${v}_$i 300 $B --queue-depth 4096 || exit 1; done
done
RSF_LIB_PATH=$PWD/ab/lib_dbase.so bash $S q64_dbase 300 $B || exit 1
for f in deep_dbase_1 deep_s94_1 deep_dbase_2 deep_s94_2 q64_dbase; do grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phases_ms_per_round'].items()}, d.get('deep_path_members_per_round'))"; done
