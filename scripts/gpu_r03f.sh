#!/bin/bash
# multi-GPU path cost (forced one-rank RCCL) with the decoration rebuild fused into the bucket
# index pass vs the separate kernel; emission A/B; SQ instruction counters of the emission
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points"
F="RSF_FORCE_SHARDED=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29523"
bash $S dist_tests 400 python -u -m pytest tests/test_gossip_gpu.py tests/test_dist_gpu.py -x -q --timeout 200 --timeout-method thread -k "two_shards or dist or rccl" && \
bash $S single_1 200 $B && \
env $F bash $S sharded_fused 200 $B && \
env $F RSF_LIB_PATH=$PWD/ab/lib_unfused.so bash $S sharded_unfused 200 $B && \
RSF_LIB_PATH=$PWD/ab/lib_nolazy.so bash $S single_nolazy 200 $B && \
RSF_LIB_PATH=$PWD/ab/lib_nopin.so bash $S single_nopin 200 $B && \
bash $S single_2 200 $B && \
bash $S pmc_emit 300 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_r03_1 -o run -- python3 bench.py --workload gossip --steps 3 --warmup 1 --no-cpu-baseline --no-vivaldi --no-extra-points
tail -2 gpurun_out/dist_tests.log
for f in single_1 sharded_fused sharded_unfused single_nolazy single_nopin single_2; do grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), 'wall/steps vs kernels:', {k: round(v,3) for k,v in d['phases_ms_per_round'].items()})"; done
