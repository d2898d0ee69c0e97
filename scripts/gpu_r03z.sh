#!/bin/bash
# bucket emission: slot words pre-encoded with (shard, bucket place) -- no division, no
# dependent wstart load in emit_kernel<true>; parity + forced one-rank sharded A/B vs HEAD
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points"
F="RSF_FORCE_SHARDED=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29523"
bash $S tests 600 python -u -m pytest tests/test_gossip_gpu.py tests/test_dist_gpu.py tests/test_dist_vivaldi_gpu.py -x -q --timeout 300 --timeout-method thread && \
for i in 1 2; do
  env $F RSF_LIB_PATH=$PWD/ab/lib_head.so bash $S shead$i 200 $B && env $F bash $S scur$i 200 $B && bash $S single$i 200 $B || exit 1
done
tail -2 gpurun_out/tests.log
for f in shead1 scur1 single1 shead2 scur2 single2; do grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phases_ms_per_round'].items()}, d.get('exchange_ok'))"; done
