#!/bin/bash
# multi-GPU path: own bucket read in place (no self copy), decorations looked up by the merge
# (RSF_BUCKET_DEC_MODE 2) vs the rebuild kernel (0), emission writing the bucket keys;
# forced one-rank timings + a kernel trace of the forced path
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points"
F="RSF_FORCE_SHARDED=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29523"
bash $S dist_tests 400 python -u -m pytest tests/test_gossip_gpu.py tests/test_dist_gpu.py -x -q --timeout 200 --timeout-method thread -k "two_shards or dist or rccl or bucket" && \
bash $S single_1 200 $B && \
env $F bash $S sharded_dec2 200 $B && \
env $F RSF_LIB_PATH=$PWD/ab/lib_dec0.so bash $S sharded_dec0 200 $B && \
env $F bash $S sharded_dec2b 200 $B && \
env $F bash $S trace_sharded 300 timeout -s KILL 250 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03g_s -o run -- python3 bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points --steps 5 --warmup 2
tail -2 gpurun_out/dist_tests.log
for f in single_1 sharded_dec2 sharded_dec0 sharded_dec2b; do grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phases_ms_per_round'].items()}, d.get('collectives_ms_per_round'), d.get('exchange_ok'))"; done
