#!/bin/bash
# rocprofv3 trace + FETCH/WRITE of the gossip round after the deferred re-queues
bash scripts/profile.sh r02l_gossip gossip --no-vivaldi
