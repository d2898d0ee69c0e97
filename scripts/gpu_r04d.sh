#!/bin/bash
# round 4: deep-queue bench points (configs[1] q64 vs depth 4096, same call), the 2M headline,
# then the Vivaldi variant A/B
S=scripts/gpu_step.sh
bash scripts/gpu_r04c.sh || exit 1
bash $S viv_ab 900 bash scripts/ab_viv4.sh vbase vown vwlate vown4
