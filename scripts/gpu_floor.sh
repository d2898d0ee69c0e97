#!/bin/bash
# merge access-pattern floor (experiments/view_floor.hip), built on the box; then a kernel
# trace of the multi-GPU code path forced on one GPU
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -w -o gpurun_out/view_floor experiments/view_floor.hip && \
bash scripts/gpu_step.sh view_floor 120 gpurun_out/view_floor && cat gpurun_out/view_floor.log && \
bash scripts/prof_sharded1.sh
