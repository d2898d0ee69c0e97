#!/bin/bash
# round 5: checker prune selects unrolled + shared histograms, compact phase grids; its split per member
S=scripts/gpu_step.sh
bash $S pytest_deep 900 python -u -m pytest tests/test_deep_queue_gpu.py tests/test_gossip_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_deep.log && ! grep -q " failed\| error" gpurun_out/pytest_deep.log || exit 1
bash $S check_prof 300 python -u experiments/check_prof.py 1000000 300 || exit 1
RSF_LIB_PATH=$PWD/abx/lib_prof.so bash $S check_prof_split 300 python -u experiments/check_prof.py 1000000 300 || exit 1
bash $S steady_stag 400 python -u experiments/steady_state.py 1000000 420 150 8704 10 stagger
