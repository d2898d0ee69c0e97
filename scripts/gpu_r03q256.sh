#!/bin/bash
# the no-drop point (configs[1] shape, queue_cap 256, 3 settle rounds): rocprofv3 trace + FETCH/WRITE
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
bash scripts/profile.sh r03f_q256 gossip --no-vivaldi --no-extra-points --members 1000000 --queue-cap 256 --settle 3
