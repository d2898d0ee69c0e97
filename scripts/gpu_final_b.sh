#!/bin/bash
# round 6 final tree, part 2: the gossip and Vivaldi profiles (kernel trace + FETCH/WRITE
# passes), the default line's multi-GPU path on one RCCL rank against the single context (same
# box, alternating, no profiler), the configs[2] shard in the reference regime, configs[3] churn
S=scripts/gpu_step.sh
bash scripts/profile.sh r06_gossip gossip --no-extra-points --no-vivaldi || exit 1
bash scripts/profile.sh r06_viv vivaldi || exit 1
for i in 1 2; do
  RSF_FORCE_SHARDED=1 bash $S sharded_$i 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port $((29541 + i)) bench.py --steps 20 --no-extra-points --no-vivaldi --no-cpu-baseline || exit 1
  bash $S single_$i 600 python -u bench.py --steps 20 --no-extra-points --no-vivaldi --no-cpu-baseline || exit 1
done
bash $S bench_2m 600 python -u bench.py --workload gossip --members 2000000 --steps 20 --warmup 3 --no-cpu-baseline --no-vivaldi --no-extra-points || exit 1
bash $S bench_churn 600 python -u bench.py --workload churn --steps 20 --warmup 3 --no-cpu-baseline || exit 1
for f in sharded_1 single_1 sharded_2 single_2 bench_2m bench_churn; do grep -h '^{' gpurun_out/$f.log | cut -c1-200; done
