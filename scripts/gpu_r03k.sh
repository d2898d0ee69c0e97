#!/bin/bash
# emit_kernel phase split with per-wave register accumulators (no contended atomics between phases)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
RSF_LIB_PATH=$PWD/ab/lib_eprof.so bash $S emit_prof 300 python3 experiments/merge_prof.py 2000000 emit
grep -E "^\{|eprof2" gpurun_out/emit_prof.log
