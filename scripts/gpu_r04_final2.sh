#!/bin/bash
# round 4 final tree: rocprofv3 kernel trace + FETCH/WRITE of the gossip round (2M shard) and
# of Vivaldi (64M), kernel trace of the configs[1] depth-4096 point, SQ instruction counters
# of the gossip round, the forced one-rank multi-GPU path beside a single-context round
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points"
F="RSF_FORCE_SHARDED=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29523"
bash $S prof_gossip 900 bash scripts/profile.sh r04_gossip gossip --no-vivaldi --no-extra-points && \
bash $S prof_viv 900 bash scripts/profile.sh r04_viv vivaldi && \
bash $S kt_deep 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04_deep_trace -o run -- python3 bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points --members 1000000 --steps 10 --queue-depth 4096 && \
bash $S kt_q64 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04_q64_trace -o run -- python3 bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points --members 1000000 --steps 10 && \
bash $S pmc_sq 600 bash scripts/pmc_sq.sh r04 --workload gossip --no-vivaldi --no-extra-points && \
bash $S single_1 200 $B && env $F bash $S sharded_1 200 $B && bash $S single_2 200 $B && env $F bash $S sharded_2 200 $B
for f in single_1 sharded_1 single_2 sharded_2; do grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phases_ms_per_round'].items()}, d.get('collectives_ms_per_round'), d.get('exchange_ok'))"; done
