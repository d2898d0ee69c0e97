#!/bin/bash
# kernel trace of the default gossip round: per-round span vs kernel-busy time and the gaps between launches
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
bash $S trace 300 timeout -s KILL 250 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/trace_r03x -o run -- python3 bench.py --workload gossip --steps 5 --warmup 1 --no-cpu-baseline --no-vivaldi --no-extra-points
python3 experiments/trace_gaps.py gpurun_out/trace_r03x/run_kernel_trace.csv merge_kernel > gpurun_out/trace_gaps_r03x.txt 2>&1
cat gpurun_out/trace_gaps_r03x.txt
