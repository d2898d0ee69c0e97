#!/bin/bash
# round-3 final measurements of the tree: GPU suite, smoke, default bench line (both halves + CPU
# baselines), rocprofv3 kernel trace + FETCH/WRITE of the gossip round, forced multi-GPU code
# path on one GPU beside a single-context round
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points"
F="RSF_FORCE_SHARDED=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29523"
bash $S pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread && \
bash $S smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" && \
bash $S bench_default 500 python -u bench.py && \
bash scripts/profile.sh r03f_gossip gossip --no-vivaldi --no-extra-points && \
bash $S single_1 200 $B && env $F bash $S sharded_1 200 $B && bash $S single_2 200 $B && env $F bash $S sharded_2 200 $B
tail -2 gpurun_out/pytest_gpu.log
for f in single_1 sharded_1 single_2 sharded_2; do grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phases_ms_per_round'].items()}, d.get('collectives_ms_per_round'), d.get('exchange_ok'))"; done
grep -h '^{' gpurun_out/bench_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['vivaldi']['value'], d['vivaldi']['roofline']['frac'])"
