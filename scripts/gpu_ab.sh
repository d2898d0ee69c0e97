#!/bin/bash
# gpu_ab.sh VARIANT... : gossip GPU tests on the default build, then A/B bench of variants
S=scripts/gpu_step.sh
bash $S pytest_gossip 400 python -u -m pytest tests/test_gossip_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "failed\|error" gpurun_out/pytest_gossip.log && exit 1
WLS=${WLS:-gossip} timeout -k 10 900 bash experiments/ab_variants.sh "$@"
