#!/bin/bash
# round 6: record decorations travel in the buckets (no receive-side rebuild) -- the bucket /
# multi-GPU parity tests, kernel traces of the default line through the multi-GPU code path on
# one rank and through the single context, then the deferred path's and the checker's
# shader-clock splits (scripts/gpu_r06k.sh)
S=scripts/gpu_step.sh
bash $S pytest_bkt 700 python -u -m pytest tests/test_dist_gpu.py tests/test_deep_queue_gpu.py tests/test_gossip_gpu.py -v -s --timeout 600 --timeout-method thread -x -k "bucket or shard or rccl or dist or two or context" || exit 1
grep -q " passed" gpurun_out/pytest_bkt.log && ! grep -q " failed\| error" gpurun_out/pytest_bkt.log || { grep -h "FAILED\|Error" gpurun_out/pytest_bkt.log | head; exit 1; }
bash scripts/gpu_r06h.sh || exit 1
python3 experiments/trace_compare.py gpurun_out/prof_sh/run_kernel_trace.csv gpurun_out/prof_single/run_kernel_trace.csv 5 | tee gpurun_out/trace_compare.txt
bash scripts/gpu_r06k.sh || exit 1
grep -h "passed\|failed" gpurun_out/pytest_bkt.log | tail -1
