#!/bin/bash
# round 6: chunked Vivaldi exchange parity, Vivaldi line, the 1M regime kernel-trace profile,
# the merge's rumor-body gather against a ring small enough for the MALL (--ring-rounds 64)
S=scripts/gpu_step.sh
bash $S pytest_viv 900 python -u -m pytest tests/test_dist_vivaldi_gpu.py tests/test_vivaldi_gpu.py tests/test_capi.py -v --timeout 600 --timeout-method thread -x || exit 1
bash $S bench_viv 600 python -u bench.py --workload vivaldi --steps 20 --warmup 3 --no-cpu-baseline || exit 1
bash scripts/profile.sh r06a_gossip gossip --no-extra-points --no-vivaldi || exit 1
for i in 1 2; do
  bash $S ring_full_$i 400 python -u bench.py --workload gossip --steps 20 --warmup 3 --no-cpu-baseline --no-vivaldi --no-extra-points || exit 1
  bash $S ring_64_$i 400 python -u bench.py --workload gossip --steps 20 --warmup 3 --no-cpu-baseline --no-vivaldi --no-extra-points --ring-rounds 64 || exit 1
done
grep -h "passed\|failed" gpurun_out/pytest_viv.log | tail -2
