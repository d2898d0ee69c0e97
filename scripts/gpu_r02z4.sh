#!/bin/bash
# merge floor at the bench's measured mix; emit_kernel shader-clock phase split (diagnostic build)
S=scripts/gpu_step.sh
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -w -o gpurun_out/view_floor experiments/view_floor.hip && \
bash $S view_floor 120 gpurun_out/view_floor && cat gpurun_out/view_floor.log && \
RSF_LIB_PATH=$PWD/ab/lib_eprof.so bash $S emit_prof 300 python3 experiments/merge_prof.py 2000000 emit && cat gpurun_out/emit_prof.log
