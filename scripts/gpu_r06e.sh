#!/bin/bash
# round 6: the default line's multi-GPU code path on one RCCL rank against the single context
# (same box, alternating), and a two-rank gloo rehearsal of bench.py --gpus 2 (both ranks on
# this GPU: the gossip regime at 250k members per rank, Vivaldi 64M with the chunked exchange)
S=scripts/gpu_step.sh
for i in 1 2; do
  RSF_FORCE_SHARDED=1 bash $S sharded_$i 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port $((29511 + i)) bench.py --steps 20 --no-extra-points --no-vivaldi --no-cpu-baseline || exit 1
  bash $S single_$i 600 python -u bench.py --steps 20 --no-extra-points --no-vivaldi --no-cpu-baseline || exit 1
done
RSF_DIST_BACKEND=gloo bash $S gloo2 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 2 --members 250000 --no-extra-points || exit 1
for f in sharded_1 single_1 sharded_2 single_2 gloo2; do grep -h '^{' gpurun_out/$f.log | cut -c1-300; done
