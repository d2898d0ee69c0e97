#!/bin/bash
# round 5: profiles of the default line's kernels (gossip in the reference regime, Vivaldi), per-class deferral split
S=scripts/gpu_step.sh
bash scripts/profile.sh r05_gossip gossip --no-extra-points --no-vivaldi || exit 1
bash scripts/profile.sh r05_viv vivaldi || exit 1
RSF_LIB_PATH=$PWD/abx/lib_prof.so bash $S deep_prof 400 python -u experiments/deep_prof.py 1000000 360 8704 150 || exit 1
RSF_LIB_PATH=$PWD/abx/lib_prof.so bash $S check_prof_split 300 python -u experiments/check_prof.py 1000000 300
