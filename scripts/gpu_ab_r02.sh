#!/bin/bash
# A/B of merge variants (timing-only experiment flags) + SQ occupancy counters of the base
S=scripts/gpu_step.sh
WLS=gossip bash $S ab 900 bash experiments/ab_variants.sh base noq norb noqrb m4 && \
bash $S sq 400 bash scripts/pmc_sq.sh base --workload gossip --no-vivaldi
