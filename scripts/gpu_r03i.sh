#!/bin/bash
# emit_kernel phase split (diagnostic build); decorations gathered from rdec (RSF_Q_DEC 0) vs kept in the queue: parity + A/B
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points"
RSF_LIB_PATH=$PWD/ab/lib_eprof.so bash $S emit_prof 300 python3 experiments/merge_prof.py 2000000 emit && \
RSF_LIB_PATH=$PWD/ab/lib_qdec0.so bash $S qdec0_tests 400 python -u -m pytest tests/test_gossip_gpu.py -x -q --timeout 200 --timeout-method thread && \
for i in 1 2; do
  bash $S def$i 200 $B && RSF_LIB_PATH=$PWD/ab/lib_qdec0.so bash $S qdec0_$i 200 $B || exit 1
done
tail -2 gpurun_out/qdec0_tests.log
for f in def1 qdec0_1 def2 qdec0_2; do grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phases_ms_per_round'].items()})"; done
