#!/bin/bash
# round 5: checker pass 1 with the first radix pass fused; its split; a kernel trace of the staggered steady state
S=scripts/gpu_step.sh
bash $S pytest_deep 900 python -u -m pytest tests/test_deep_queue_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "staggered or steady or check or churn or bench_shape or ticks" || exit 1
grep -q " passed" gpurun_out/pytest_deep.log && ! grep -q " failed\| error" gpurun_out/pytest_deep.log || exit 1
bash $S check_prof 300 python -u experiments/check_prof.py 1000000 300 || exit 1
RSF_LIB_PATH=$PWD/abx/lib_prof.so bash $S check_prof_split 300 python -u experiments/check_prof.py 1000000 300 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash $S trace_stag 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_stag -o run -- python3 experiments/steady_state.py 1000000 360 150 8704 10 stagger || exit 1
python3 experiments/trace_last.py $(ls gpurun_out/tr_stag/*/run_kernel_trace.csv gpurun_out/tr_stag/run_kernel_trace.csv 2>/dev/null | head -1) 20 > gpurun_out/trace_stag_last20.txt 2>&1
