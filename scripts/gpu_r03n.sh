#!/bin/bash
# PC sampling of the gossip round (where emit / merge spend their issue slots)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
bash $S pcs_list 60 timeout -s KILL 50 rocprofv3 -L && \
bash $S pcs 240 timeout -s KILL 200 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 --output-format csv -d gpurun_out/pcs_r03n -o run -- python3 bench.py --workload gossip --members 1000000 --steps 4 --warmup 1 --no-cpu-baseline --no-vivaldi --no-extra-points
grep -i -B2 -A12 "pc_sampl\|PC sampling" gpurun_out/pcs_list.log | head -60
ls -la gpurun_out/pcs_r03n 2>/dev/null
