#!/bin/bash
# round 6: merge_kernel receivers per wave (RSF_MERGE_PER_WAVE, 8 by default, tuned at round 4 on
# the 2M 64-slot shard) re-measured in the reference regime at 1M: same-box A/B of 4 and 16
bash scripts/ab.sh abx 2 gossip default mpw4 mpw16 || exit 1
