#!/bin/bash
# emission: queue-major picks + v_mbcnt / inverse-ballot lane masks (working tree) vs HEAD;
# parity of the working tree; SQ instruction mix; phase split
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 -u bench.py --workload gossip --no-vivaldi --no-cpu-baseline --no-extra-points"
P="python3 bench.py --workload gossip --steps 3 --warmup 1 --no-cpu-baseline --no-vivaldi --no-extra-points"
bash $S tests 500 python -u -m pytest tests/test_gossip_gpu.py tests/test_dist_gpu.py tests/test_snapshot_gpu.py tests/test_pushpull_gpu.py tests/test_reap_gpu.py -x -q --timeout 200 --timeout-method thread && \
for i in 1 2; do
  RSF_LIB_PATH=$PWD/ab/lib_head.so bash $S head$i 200 $B && bash $S cur$i 200 $B || exit 1
done
bash $S pmc_a 200 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH --output-format csv -d gpurun_out/pmc_r03q_a -o run -- $P
tail -2 gpurun_out/tests.log
for f in head1 cur1 head2 cur2; do grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phases_ms_per_round'].items()})"; done
python3 - <<'PY'
import csv, collections
rows=list(csv.DictReader(open('gpurun_out/pmc_r03q_a/run_counter_collection.csv')))
agg=collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    k=r['Kernel_Name']
    if 'emit_kernel' in k or 'merge_kernel<false' in k:
        kk='emit' if 'emit' in k else 'merge'
        agg[kk][r['Counter_Name']]+=float(r['Counter_Value'])
for kk,d in agg.items():
    w=d['SQ_WAVES']; print(kk, {c: round(v/w,1) for c,v in d.items() if c!='SQ_WAVES'})
PY
RSF_LIB_PATH=$PWD/ab/lib_eprof.so bash $S emit_prof 300 python3 experiments/merge_prof.py 2000000 emit; grep -E "^\{|eprof2" gpurun_out/emit_prof.log | tail -6
