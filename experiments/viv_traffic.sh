#!/bin/bash
# Vivaldi round-kernel HBM traffic: the ablation driver under FETCH_SIZE and WRITE_SIZE
# passes (separate, per MI355X_MICROARCH.md), plus a plain timing run.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
D=gpurun_out/viv_traffic; mkdir -p $D
N=${1:-64000000}
timeout -k 10 240 python3 experiments/viv_ablate.py $N > $D/times.json 2> $D/times.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- python3 experiments/viv_ablate.py $N > $D/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- python3 experiments/viv_ablate.py $N > $D/write.log 2>&1 || exit $?
python3 experiments/viv_traffic.py $D | tee $D/summary.txt
