#!/bin/bash
# round 6: the queue heads without per-item decorations (an intent's record decoration read from
# the rumor table when it is sent) and 8-B pending entries -- the whole GPU suite on that build
# (abx/lib_hdec.so through RSF_LIB_PATH), then a same-box A/B against the current tree
S=scripts/gpu_step.sh
RSF_LIB_PATH=$PWD/abx/lib_hdec.so bash $S pytest_hdec 900 python -u -m pytest tests -m gpu -v -s --timeout 800 --timeout-method thread -x || exit 1
grep -q " passed" gpurun_out/pytest_hdec.log && ! grep -q " failed\| error" gpurun_out/pytest_hdec.log || { grep -h "FAILED\|Error" gpurun_out/pytest_hdec.log | head; exit 1; }
bash scripts/ab.sh abx 2 gossip nodec hdec || exit 1
grep -h "passed\|failed" gpurun_out/pytest_hdec.log | tail -2
