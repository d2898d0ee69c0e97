#!/bin/bash
# diagnostic: guard zones around big_ids / stage_dec / the sort's storage, in the clean layout
# (library probed first), bench workload at 1M; then the production build's GPU suite
RSF_LIB_PATH=$PWD/ab/lib_zones.so timeout -k 10 200 python3 -u experiments/cfg1_checks.py 1000000 4096 0 15 bench nosync torchstream torchfirst > gpurun_out/zones.log 2>&1
echo "zones rc=$?"; grep "guard zones\|^ptrs" gpurun_out/zones.log | cut -c1-400; tail -1 gpurun_out/zones.log | cut -c1-200
bash scripts/gpu_step.sh pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -1 gpurun_out/pytest_gpu.log
