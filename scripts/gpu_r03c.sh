#!/bin/bash
# round 3 profiles: rocprofv3 kernel trace of the default gossip leg (2M, lazy emission) and of
# the multi-GPU code path forced on one GPU; emit phase split with and without the lazy re-rank
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
bash $S prof_g 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03g_trace -o run -- python3 bench.py --workload gossip --steps 5 --warmup 1 --no-cpu-baseline --no-vivaldi && \
RSF_FORCE_SHARDED=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29523 bash $S prof_s1 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03s1_trace -o run -- python3 bench.py --workload gossip --steps 5 --warmup 1 --no-cpu-baseline --no-vivaldi && \
RSF_LIB_PATH=$PWD/ab/lib_eprof.so bash $S eprof 300 python3 experiments/merge_prof.py 2000000 emit && \
RSF_LIB_PATH=$PWD/ab/lib_eprof_nolazy.so bash $S eprof_nolazy 300 python3 experiments/merge_prof.py 2000000 emit
cat gpurun_out/eprof.log gpurun_out/eprof_nolazy.log | grep '^{'
