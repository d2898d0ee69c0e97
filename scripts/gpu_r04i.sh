#!/bin/bash
S=scripts/gpu_step.sh
bash $S dprof30 300 env RSF_LIB_PATH=$PWD/ab/lib_dprof.so python -u experiments/deep_prof.py 1000000 30
