#!/bin/bash
# round 3 profiles and A/B: emission variants (default = lazy re-rank + speculative pending
# load; nospec; nolazy) at 2M, rocprofv3 kernel traces of the default gossip leg and of the
# multi-GPU code path forced on one GPU, emit phase split
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points"
bash $S ab_def1 200 $B && \
RSF_LIB_PATH=$PWD/ab/lib_nospec.so bash $S ab_nospec 200 $B && \
bash $S ab_def2 200 $B && \
bash $S prof_g 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03g_trace -o run -- python3 bench.py --workload gossip --steps 5 --warmup 1 --no-cpu-baseline --no-vivaldi --no-extra-points && \
RSF_FORCE_SHARDED=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29523 bash $S prof_s1 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03s1_trace -o run -- python3 bench.py --workload gossip --steps 5 --warmup 1 --no-cpu-baseline --no-vivaldi --no-extra-points && \
RSF_LIB_PATH=$PWD/ab/lib_eprof.so bash $S eprof 300 python3 experiments/merge_prof.py 2000000 emit
for f in ab_def1 ab_nospec ab_def2; do grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phases_ms_per_round'].items()})"; done
grep '^{' gpurun_out/eprof.log
