#!/bin/bash
# round 4: deep-path diagnostics (deferral reasons, phase cycles) + a kernel trace of the deep bench
S=scripts/gpu_step.sh
export RSF_LIB_PATH_SAVE=
bash $S dprof12 300 env RSF_LIB_PATH=$PWD/ab/lib_dprof.so python -u experiments/deep_prof.py 1000000 12 || exit 1
bash $S dprof30 300 env RSF_LIB_PATH=$PWD/ab/lib_dprof.so python -u experiments/deep_prof.py 1000000 30 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash $S ktrace_deep 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_deep -o kt -- python3 bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points --members 1000000 --queue-depth 4096 --steps 10
