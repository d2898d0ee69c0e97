#!/bin/bash
# round 4: kernel trace of the q64 and depth-4096 configs[1] points (same box)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points --members 1000000 --steps 10"
bash $S kt_q64 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_q64 -o kt -- $B || exit 1
bash $S kt_deep 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_deep -o kt -- $B --queue-depth 4096
