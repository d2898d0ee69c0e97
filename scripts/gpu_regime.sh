#!/bin/bash
# gpu_regime.sh MODE [ARGS]: the reference-regime probes on one GPU, each
# step under its own time limit (gpu_step.sh), logs in gpurun_out/.
#   parity          the deep-queue and gossip GPU suites (stops the call on a failure)
#   steady [MODE]   experiments/steady_state.py: 1M members, depth 8704, ticks every 150 rounds
#                   (MODE inround (default), stagger or sync)
#   checker         experiments/check_prof.py: one tick over all 1M members after 300 rounds
#   deferred        experiments/deep_prof.py in the regime (on abx/lib_prof.so, a -DRSF_DEEP_PROF=1
#                   build from experiments/build_variants.sh)
#   ab V...         same-box A/B of abx/lib_V.so against the in-tree build, steady state,
#                   alternating twice; rounds 350-380 of each run in gpurun_out/ab.txt
#   anatomy         experiments/queue_anatomy.py and the emit/merge overlap probe
S=scripts/gpu_step.sh
mode=$1; shift
case $mode in
  parity)
    bash $S pytest_deep 900 python -u -m pytest tests/test_deep_queue_gpu.py tests/test_gossip_gpu.py -m gpu -x -q \
      --timeout 300 --timeout-method thread || exit 1
    grep -q " passed" gpurun_out/pytest_deep.log && ! grep -q " failed\| error" gpurun_out/pytest_deep.log ;;
  steady)
    bash $S steady 400 python -u experiments/steady_state.py 1000000 400 150 8704 10 "${1:-inround}" ;;
  checker)
    bash $S checker 300 python -u experiments/check_prof.py 1000000 300 ;;
  deferred)
    RSF_LIB_PATH=$PWD/abx/lib_prof.so bash $S deferred 400 python -u experiments/deep_prof.py 1000000 360 8704 150 ;;
  ab)
    for v in default "$@" default "$@"; do
      lib=""; [ "$v" != default ] && lib="RSF_LIB_PATH=$PWD/abx/lib_$v.so"
      env $lib bash $S ss_$v 300 python -u experiments/steady_state.py 1000000 380 150 8704 10 inround || exit 1
      grep '"round": 3[5-8]0' gpurun_out/ss_$v.log | cut -c1-60 | sed "s/^/$v /" >> gpurun_out/ab.txt
    done ;;
  anatomy)
    bash $S anatomy 300 python -u experiments/queue_anatomy.py 1000000 110 64 && \
    bash $S overlap 300 python -u experiments/overlap_probe.py 1000000 20 ;;
  *) echo "unknown mode $mode"; exit 2 ;;
esac
