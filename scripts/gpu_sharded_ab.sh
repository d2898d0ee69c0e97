#!/bin/bash
# same-box A/B of abx/lib_V.so against the in-tree build on the forced one-rank multi-GPU path
# (the default line's gossip leg in the reference regime); one summary line per run in gpurun_out/ab_sharded.txt
S=scripts/gpu_step.sh
i=0
for v in default "$@" default "$@"; do
  i=$((i+1))
  lib=""; [ "$v" != default ] && lib="RSF_LIB_PATH=$PWD/abx/lib_$v.so"
  env $lib RSF_FORCE_SHARDED=1 bash $S sh_${v}_$i 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port $((29520 + i)) bench.py --steps 10 --no-extra-points --no-vivaldi --no-cpu-baseline || exit 1
  grep -h '^{' gpurun_out/sh_${v}_$i.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.readline()); p = d['phases_ms_per_round']
print('$v', round(d['ms_per_step'], 3), {k.split()[0]: round(x, 3) for k, x in p.items()})" >> gpurun_out/ab_sharded.txt
done
