#!/bin/bash
# gpu_probe.sh: the steady-state queue experiment and the emit/merge co-scheduling probe
S=scripts/gpu_step.sh
bash $S overlap 300 python -u experiments/overlap_probe.py 1000000 20 && \
bash $S steady 600 python -u experiments/steady_state.py 1000000 460 150 4096 10
