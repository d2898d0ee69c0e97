#!/bin/bash
# round 5: checker pass 2 fills holes (only what moves); parity (deep + gossip suites), tick A/B against the compaction
S=scripts/gpu_step.sh
bash $S pytest_deep 900 python -u -m pytest tests/test_deep_queue_gpu.py tests/test_gossip_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_deep.log && ! grep -q " failed\| error" gpurun_out/pytest_deep.log || exit 1
for v in default compact default compact; do
  lib=""; [ "$v" != default ] && lib="RSF_LIB_PATH=$PWD/abx/lib_$v.so"
  env $lib bash $S chk_$v 300 python -u experiments/check_prof.py 1000000 300 || exit 1
  grep -h '^{' gpurun_out/chk_$v.log | sed "s/^/$v /" >> gpurun_out/ab_hole.txt
done
