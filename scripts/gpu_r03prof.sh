#!/bin/bash
# final tree: Vivaldi rocprofv3 trace + FETCH/WRITE (64M), and a kernel trace of the forced one-rank multi-GPU round
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
bash scripts/profile.sh r03f_viv vivaldi && \
RSF_FORCE_SHARDED=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29523 bash $S trace_sharded 300 timeout -s KILL 250 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03f_sharded1 -o run -- python3 bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points --steps 5 --warmup 1
python3 experiments/trace_gaps.py gpurun_out/prof_r03f_sharded1/run_kernel_trace.csv merge_kernel > gpurun_out/sharded1_gaps.txt 2>&1
ls gpurun_out
