#!/bin/bash
# merge_kernel / emit_kernel shader-clock phase profiles (diagnostic builds) at 2M members
S=scripts/gpu_step.sh
RSF_LIB_PATH=$PWD/ab/lib_prof.so bash $S merge_prof 300 python3 experiments/merge_prof.py 2000000 && \
RSF_LIB_PATH=$PWD/ab/lib_eprof.so bash $S emit_prof 300 python3 experiments/merge_prof.py 2000000 emit
