#!/bin/bash
# round 6: the bucket path's receiver keys written in sorted order by grp_index_kernel (not
# scattered from the emission) and bucket_index_kernel on 32-bit indices -- the bucket /
# multi-GPU parity tests on that build (abx/lib_bk.so), then the forced one-rank multi-GPU line
# with and without it against the single context, same box, alternating
S=scripts/gpu_step.sh
RSF_LIB_PATH=$PWD/abx/lib_bk.so bash $S pytest_bkt 700 python -u -m pytest tests/test_dist_gpu.py tests/test_deep_queue_gpu.py tests/test_gossip_gpu.py -v -s --timeout 600 --timeout-method thread -x -k "bucket or shard or rccl or dist or two or context" || exit 1
grep -q " passed" gpurun_out/pytest_bkt.log && ! grep -q " failed\| error" gpurun_out/pytest_bkt.log || { grep -h "FAILED\|Error" gpurun_out/pytest_bkt.log | head; exit 1; }
for i in 1 2; do
  RSF_FORCE_SHARDED=1 bash $S sh_base_$i 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port $((29561 + i)) bench.py --steps 20 --no-extra-points --no-vivaldi --no-cpu-baseline || exit 1
  RSF_LIB_PATH=$PWD/abx/lib_bk.so RSF_FORCE_SHARDED=1 bash $S sh_bk_$i 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port $((29571 + i)) bench.py --steps 20 --no-extra-points --no-vivaldi --no-cpu-baseline || exit 1
  RSF_LIB_PATH=$PWD/abx/lib_bk.so bash $S single_bk_$i 600 python -u bench.py --steps 20 --no-extra-points --no-vivaldi --no-cpu-baseline || exit 1
done
for f in sh_base_1 sh_bk_1 single_bk_1 sh_base_2 sh_bk_2 single_bk_2; do
  grep -h '^{' gpurun_out/$f.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.readline()); p = d['phases_ms_per_round']
print('$f', round(d['ms_per_step'], 3), {k.split()[0]: round(x, 3) for k, x in p.items()})"
done
grep -h "passed\|failed" gpurun_out/pytest_bkt.log | tail -1
