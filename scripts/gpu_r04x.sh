#!/bin/bash
# round 4: select over the used key registers only (rn) vs all (base), same box x2; deep tests;
# Vivaldi profile of the final tree
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
bash $S deep_tests 900 python -u -m pytest tests/test_deep_queue_gpu.py -m gpu -q -x --timeout 600 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/deep_tests.log || exit 1
bash $S dprof30 300 env RSF_LIB_PATH=$PWD/ab/lib_dprof9.so python -u experiments/deep_prof.py 1000000 30 || exit 1
B="python3 -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points --members 1000000"
for i in 1 2; do
  for v in rn base; do RSF_LIB_PATH=$PWD/ab/lib_$v.so bash $S deep_${v}_$i 300 $B --queue-depth 4096 || exit 1; done
done
for f in deep_rn_1 deep_base_1 deep_rn_2 deep_base_2; do grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), round(d['phases_ms_per_round']['emit_kernel'],3))"; done
bash $S prof_viv 900 bash scripts/profile.sh r04b_viv vivaldi
