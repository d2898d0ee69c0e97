#!/bin/bash
# pmc_sq.sh TAG [bench args]: SQ instruction-mix / stall counters of the bench's kernels,
# two separate --pmc passes (8 SQ counters max per pass), kernel-trace only.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
tag=$1; shift
args="--steps 3 --warmup 1 --no-cpu-baseline $*"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"
i=1
for P in "$P1" "$P2"; do
  timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_${tag}_$i -o run -- python3 bench.py $args > gpurun_out/pmc_${tag}_$i.log 2>&1 || exit $?
  i=$((i+1))
done
echo "pmc $tag done"
