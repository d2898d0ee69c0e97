#!/bin/bash
# rocprofv3 kernel trace of the multi-GPU gossip code path forced on one GPU (one RCCL rank)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export RSF_FORCE_SHARDED=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29523
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sharded1_trace -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_sharded1_trace.log 2>&1
