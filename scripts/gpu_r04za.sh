#!/bin/bash
# round 4: Vivaldi pipe kernel at 128-thread blocks: Vivaldi GPU tests, then the rocprofv3 profile
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
bash $S viv_tests 900 python -u -m pytest tests/test_vivaldi_gpu.py tests/test_dist_vivaldi_gpu.py tests/test_probe_gpu.py tests/test_codec_gpu.py -m gpu -q -x --timeout 600 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/viv_tests.log || exit 1
bash $S prof_viv 900 bash scripts/profile.sh r04c_viv vivaldi
tail -1 gpurun_out/viv_tests.log
