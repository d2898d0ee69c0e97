#!/bin/bash
# gpu_step.sh NAME TIMEOUT CMD... : runs one GPU step under its own time limit,
# logs to gpurun_out/NAME.log, and aborts the whole call on a fault/abort/timeout
# (exit 124/134/137/139) so nothing else touches the GPU after it.
name=$1; shift; lim=$1; shift
mkdir -p gpurun_out
echo "== $name: $*" | tee -a gpurun_out/steps.log
timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
tail -n 5 "gpurun_out/$name.log"
case $rc in
  124|134|137|139) echo "FATAL step $name rc=$rc: stopping" ; exit 99 ;;
esac
exit 0
