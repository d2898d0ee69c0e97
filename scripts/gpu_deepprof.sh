#!/bin/bash
# gpu_deepprof.sh SETTLE...: experiments/deep_prof.py on the RSF_DEEP_PROF=1 build (abx/lib_prof.so)
S=scripts/gpu_step.sh
for st in "$@"; do
  RSF_LIB_PATH=$PWD/abx/lib_prof.so bash $S deepprof_$st 300 python -u experiments/deep_prof.py 1000000 $st || exit 1
done
