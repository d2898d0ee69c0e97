#!/bin/bash
# gpu_anatomy.sh: deep-queue anatomy and deferral profile at the bench workload (1M members)
S=scripts/gpu_step.sh
bash $S anatomy_110 300 python -u experiments/queue_anatomy.py 1000000 110 64 && \
RSF_LIB_PATH=$PWD/abx/lib_prof.so bash $S deepprof_110 300 python -u experiments/deep_prof.py 1000000 110
