#!/bin/bash
# Round-1 refresh: PMC calibration (incl. non-temporal shapes), rocprofv3 trace + FETCH/WRITE
# passes of the Vivaldi and gossip benches, then the default bench lines (with CPU baselines).
S=scripts/gpu_step.sh
bash $S pmc_calib 300 bash experiments/pmc_calib.sh && \
bash $S prof_viv 600 bash scripts/profile.sh viv_r01c vivaldi && \
bash $S prof_gossip 600 bash scripts/profile.sh gossip_r01c gossip && \
bash $S bench_default 400 python -u bench.py && \
bash $S bench_vivaldi 400 python -u bench.py --workload vivaldi
