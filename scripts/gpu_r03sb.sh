#!/bin/bash
# group sort: rocPRIM onesweep 8 bits per pass (tuned default) vs 11 / 7 bits, 6M pairs x 21-bit keys
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
S=scripts/gpu_step.sh
bash $S sort_bits 120 ./experiments/sort_bits
cat gpurun_out/sort_bits.log
