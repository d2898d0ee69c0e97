#!/bin/bash
# queue_cap > 64 diagnosis: every parameter set, and the first departing round in detail
S=scripts/gpu_step.sh
bash $S q4_all 400 python -u -m pytest tests/test_gossip_gpu.py -v --timeout 200 --timeout-method thread -k "queue_cap" ; \
bash $S q4_diff 300 python -u experiments/q4_diff.py 256 192 0.05 6000
grep -E "PASS|FAIL" gpurun_out/q4_all.log | head; cat gpurun_out/q4_diff.log | tail -30
