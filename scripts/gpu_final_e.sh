#!/bin/bash
# round 6 final tree: the gossip profile (kernel trace + FETCH/WRITE passes) of the default line
bash scripts/profile.sh r06d_gossip gossip --no-extra-points --no-vivaldi || exit 1
grep -h '^{' gpurun_out/prof_r06d_gossip_trace.log | cut -c1-200
