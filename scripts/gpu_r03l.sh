#!/bin/bash
# SQ instruction mix of emit_kernel / merge_kernel (two counter passes, kernel filter by name in post)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 bench.py --workload gossip --steps 3 --warmup 1 --no-cpu-baseline --no-vivaldi --no-extra-points"
bash $S pmc_a 200 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH --output-format csv -d gpurun_out/pmc_r03l_a -o run -- $B && \
bash $S pmc_b 200 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU --output-format csv -d gpurun_out/pmc_r03l_b -o run -- $B
find gpurun_out/pmc_r03l_a gpurun_out/pmc_r03l_b -name "*counter_collection.csv" | head
