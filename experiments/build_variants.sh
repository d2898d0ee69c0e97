#!/bin/bash
# Builds libruserf_amd variants into experiments/libs/ for A/B timing
# (load one with RSF_LIB_PATH=...).  Usage: build_variants.sh name "-DFLAG=.. ..." ...
set -e
cd "$(dirname "$0")/.."
CS=ruserf_amd/csrc
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -Wno-unused-value -Wno-unused-result"
mkdir -p experiments/libs
while [ $# -gt 1 ]; do
  name=$1; defs=$2; shift 2
  d=experiments/libs/build_$name; mkdir -p $d
  for s in capi vivaldi gossip codec coalesce swim intern; do /opt/rocm/bin/hipcc $F $defs -c $CS/$s.hip -o $d/$s.o & done; wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o experiments/libs/lib_$name.so $d/*.o
  echo built $name
done
