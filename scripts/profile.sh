#!/bin/bash
# profile.sh TAG WORKLOAD [extra bench args]: rocprofv3 kernel trace + stats, then
# FETCH_SIZE and WRITE_SIZE in separate passes (MI355X_MICROARCH.md: they do not
# fit one pass).  Outputs under gpurun_out/prof_<TAG>_*.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
tag=$1; wl=$2; shift 2
args="--workload $wl --steps 5 --warmup 1 --no-cpu-baseline $*"
set -o pipefail
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_trace -o run -- python3 bench.py $args > gpurun_out/prof_${tag}_trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_${tag}_fetch -o run -- python3 bench.py $args > gpurun_out/prof_${tag}_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_${tag}_write -o run -- python3 bench.py $args > gpurun_out/prof_${tag}_write.log 2>&1 || exit $?
echo "profile $tag done"
