#!/bin/bash
# Vivaldi: as_secs_f64 by multiply + FMA correction (exact over all nanos), filter median on
# the integers then one conversion; parity + A/B vs HEAD at 64M
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
B="python3 -u bench.py --workload vivaldi --steps 10 --warmup 2 --no-cpu-baseline"
bash $S tests 600 python -u -m pytest tests/test_vivaldi_gpu.py tests/test_codec_gpu.py tests/test_probe_gpu.py tests/test_dist_vivaldi_gpu.py tests/test_swim_gpu.py -x -q --timeout 300 --timeout-method thread && \
for i in 1 2 3; do
  RSF_LIB_PATH=$PWD/ab/lib_vhead.so bash $S vhead$i 200 $B && bash $S vcur$i 200 $B || exit 1
done
tail -2 gpurun_out/tests.log
for f in vhead1 vcur1 vhead2 vcur2 vhead3 vcur3; do grep -h '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline',{}); print('$f', d['value'], round(d['ms_per_step'],3), r.get('avg_launch_ms'), r.get('frac'))"; done
