#!/bin/bash
# Builds libruserf_amd variants into $AB (default abx/: git-ignored, travels to the GPU box; delete it after the A/B) for A/B
# timing within one gpurun call (load one with RSF_LIB_PATH=$PWD/abx/lib_NAME.so).
# REV=<rev> builds the source as of that git revision instead of the working tree.
# Only one source file is rebuilt with the extra defines (SRC=gossip by default, or vivaldi);
# the other objects come from the main build (make -C ruserf_amd/csrc first).
# Usage: build_variants.sh name "-DFLAG=.. ..." ...
set -e
cd "$(dirname "$0")/.."
CS=ruserf_amd/csrc
SRCF=${SRC:-gossip}
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -Wno-unused-value -Wno-unused-result"
AB=${AB:-abx}; mkdir -p $AB
while [ $# -gt 1 ]; do
  name=$1; defs=$2; shift 2
  d=$AB/build_$name; mkdir -p $d
  src=$CS/$SRCF.hip
  if [ -n "$REV" ]; then
    rm -rf $d/src && mkdir -p $d/src && git archive "$REV" ruserf_amd/csrc include | tar -x -C $d/src
    src=$d/src/ruserf_amd/csrc/$SRCF.hip
  fi
  /opt/rocm/bin/hipcc $F $defs -c $src -o $d/$SRCF.o
  objs=""
  for s in capi vivaldi gossip codec coalesce swim intern; do
    [ "$s" = "$SRCF" ] && objs="$objs $d/$s.o" || objs="$objs $CS/build/$s.o"
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $AB/lib_$name.so $objs
  echo built $name
done
