#!/bin/bash
# round 5: sealed pulls (recent mode pulls the sealed items below the head's largest key in); parity, regime, split
S=scripts/gpu_step.sh
bash $S pytest_deep 900 python -u -m pytest tests/test_deep_queue_gpu.py tests/test_gossip_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_deep.log && ! grep -q " failed\| error" gpurun_out/pytest_deep.log || exit 1
bash $S steady_inround 400 python -u experiments/steady_state.py 1000000 400 150 8704 10 inround || exit 1
RSF_LIB_PATH=$PWD/abx/lib_prof.so bash $S deep_prof 400 python -u experiments/deep_prof.py 1000000 360 8704 150
