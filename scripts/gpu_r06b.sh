#!/bin/bash
# round 6: packed intent tails -- device memory, the GPU suite (regime test included), same-box
# A/B against the 16-B tail build (abx/lib_old.so) at the 1M regime line, a 2M regime attempt
S=scripts/gpu_step.sh
bash $S meminfo 120 python -c "import torch; f, t = torch.cuda.mem_get_info(); print('free', f, 'total', t, t / 2**30, 'GiB')" || exit 1
bash $S pytest_gpu 1100 python -u -m pytest tests -m gpu -v -s --timeout 1500 --timeout-method thread -x || exit 1
bash scripts/ab.sh abx 2 gossip old default || exit 1
bash $S bench_2m 600 python -u bench.py --workload gossip --members 2000000 --steps 20 --warmup 3 --no-cpu-baseline --no-vivaldi --no-extra-points
grep -h "passed\|failed" gpurun_out/pytest_gpu.log | tail -2
bash $S bench_churn 600 python -u bench.py --workload churn --steps 20 --warmup 3 --no-cpu-baseline
grep -h '^{' gpurun_out/bench_churn.log | cut -c1-600
