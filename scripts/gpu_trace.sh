#!/bin/bash
# quick kernel trace of a bench configuration: gpu_trace.sh TAG [bench args]
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
tag=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr_$tag -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/tr_$tag.log 2>&1
