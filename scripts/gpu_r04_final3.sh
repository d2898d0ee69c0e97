#!/bin/bash
# round 4 final tree (after the deferred-path select changes): GPU suite, smoke, default bench
# line, kernel trace of the configs[1] depth-4096 and q64 points
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
bash $S pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread && \
bash $S smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" && \
bash $S bench_default 700 python -u bench.py && \
bash $S kt_deep 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04f_deep_trace -o run -- python3 bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points --members 1000000 --steps 10 --queue-depth 4096 && \
bash $S kt_q64 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04f_q64_trace -o run -- python3 bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points --members 1000000 --steps 10
tail -2 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/smoke.log
