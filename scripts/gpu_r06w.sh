#!/bin/bash
# round 6: the Vivaldi pipe kernel's block size re-measured at 64M (RSF_VIV_BLOCK 128 by default;
# 64 and 192): same-box A/B of the Vivaldi line
bash scripts/ab.sh abx 2 vivaldi default vb64 vb192 || exit 1
