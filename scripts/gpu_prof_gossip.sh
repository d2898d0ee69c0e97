#!/bin/bash
# rocprofv3 kernel trace + FETCH/WRITE passes and the SQ counter passes of the default gossip bench
set -o pipefail
timeout -k 10 900 bash scripts/profile.sh gossip_r01 gossip && \
timeout -k 10 600 bash scripts/pmc_sq.sh gossip_r01 --workload gossip
