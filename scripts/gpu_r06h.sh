#!/bin/bash
# round 6: kernel traces of the default line through the multi-GPU code path on one rank
# (RSF_FORCE_SHARDED=1, RCCL, world 1) and through the single context, to split the bucket
# path's one-rank overhead by kernel
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
args="--steps 5 --warmup 1 --no-extra-points --no-vivaldi --no-cpu-baseline"
RSF_FORCE_SHARDED=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29557 \
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sh -o run -- python3 bench.py $args > gpurun_out/prof_sh.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_single -o run -- python3 bench.py $args > gpurun_out/prof_single.log 2>&1 || exit $?
grep -h '^{' gpurun_out/prof_sh.log gpurun_out/prof_single.log | cut -c1-200
