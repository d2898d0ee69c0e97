#!/bin/bash
# configs[1] (1M members on one GPU, 4096 subjects) as a bench line beside the default 2M shard
S=scripts/gpu_step.sh
bash $S bench_1m 300 python -u bench.py --workload gossip --members 1000000 --steps 32 --warmup 3 --no-cpu-baseline --no-vivaldi
grep '^{' gpurun_out/bench_1m.log | cut -c1-400
