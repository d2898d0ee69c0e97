#!/bin/bash
# round 6: shader-clock splits of the deferred path and of the checker's prune on the current
# tree (packed intent tail, no decorations in the deferred path's LDS), reference regime, 1M
S=scripts/gpu_step.sh
RSF_LIB_PATH=$PWD/abx/lib_dprof.so bash $S deep_prof 400 python -u experiments/deep_prof.py 1000000 330 8704 150 || exit 1
RSF_LIB_PATH=$PWD/abx/lib_dprof.so bash $S check_prof 400 python -u experiments/check_prof.py 1000000 300 || exit 1
grep -h '^{' gpurun_out/deep_prof.log gpurun_out/check_prof.log | cut -c1-3000
