#!/bin/bash
# 32-bit budget arithmetic in the picks: parity + A/B vs HEAD at 2M (queue_cap 64) and 1M (queue_cap 256)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points"
B4="python3 -u bench.py --workload gossip --members 1000000 --queue-cap 256 --settle 3 --no-vivaldi --no-cpu-baseline --no-extra-points"
bash $S tests 600 python -u -m pytest tests/test_gossip_gpu.py tests/test_dist_gpu.py tests/test_snapshot_gpu.py tests/test_pushpull_gpu.py tests/test_reap_gpu.py -x -q --timeout 300 --timeout-method thread && \
for i in 1 2; do
  RSF_LIB_PATH=$PWD/ab/lib_head.so bash $S head$i 200 $B && bash $S cur$i 200 $B && \
  RSF_LIB_PATH=$PWD/ab/lib_head.so bash $S q4head$i 200 $B4 && bash $S q4cur$i 200 $B4 || exit 1
done
tail -2 gpurun_out/tests.log
for f in head1 cur1 head2 cur2 q4head1 q4cur1 q4head2 q4cur2; do grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phases_ms_per_round'].items()})"; done
bash $S pmc_a 200 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH --output-format csv -d gpurun_out/pmc_r03aa -o run -- python3 bench.py --workload gossip --steps 3 --warmup 1 --no-cpu-baseline --no-vivaldi --no-extra-points
python3 - <<'PY'
import csv, collections
rows=list(csv.DictReader(open('gpurun_out/pmc_r03aa/run_counter_collection.csv')))
agg=collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    if 'emit_kernel' in r['Kernel_Name']:
        agg['emit'][r['Counter_Name']]+=float(r['Counter_Value'])
for kk,d in agg.items():
    w=d['SQ_WAVES']; print(kk, {c: round(v/w,1) for c,v in d.items() if c!='SQ_WAVES'})
PY
