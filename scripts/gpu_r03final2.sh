#!/bin/bash
# final tree: GPU suite, smoke, default bench line
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
bash $S pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread && \
bash $S smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" && \
bash $S bench_default 500 python -u bench.py
tail -2 gpurun_out/pytest_gpu.log
grep -h '^{' gpurun_out/bench_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['phases_ms_per_round'], d['vivaldi']['value'], d['vivaldi']['roofline']['frac'])"
