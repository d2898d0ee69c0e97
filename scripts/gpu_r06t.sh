#!/bin/bash
# round 6: check_stream_kernel's unrolls re-measured on the packed tail (pass 1 loads in flight
# RSF_CHK_U1 = 32 by default, pass 2 items per thread RSF_CHK_U2 = 16): same-box A/B
bash scripts/ab.sh abx 2 gossip default u1_16 u2_8 u2_32 || exit 1
