#!/bin/bash
# round 6: sector-aligned 12-B view rows -- the GPU suite, same-box A/B against the 16-B layout
# (abx/lib_old.so: 16-B tails and views) and the unaligned 12-B views (abx/lib_p12.so), the 2M
# regime point, the churn bench bounded and in the regime
S=scripts/gpu_step.sh
bash $S pytest_gpu 1100 python -u -m pytest tests -m gpu -v -s --timeout 1500 --timeout-method thread -x || exit 1
bash scripts/ab.sh abx 2 gossip old p12 default || exit 1
bash $S bench_2m 600 python -u bench.py --workload gossip --members 2000000 --steps 20 --warmup 3 --no-cpu-baseline --no-vivaldi --no-extra-points
bash $S churn_q64 600 python -u bench.py --workload churn --steps 20 --warmup 3 --no-cpu-baseline --queue-depth 0
bash $S churn_regime 600 python -u bench.py --workload churn --steps 20 --warmup 3 --no-cpu-baseline
grep -h "passed\|failed" gpurun_out/pytest_gpu.log | tail -2
