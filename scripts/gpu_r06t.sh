#!/bin/bash
# round 6: tunables re-measured in the reference regime at 1M (same-box A/B): check_stream_kernel's
# unrolls on the packed tail (pass 1 loads in flight RSF_CHK_U1 = 32, pass 2 items per thread
# RSF_CHK_U2 = 16), the deferred path's reserve (RSF_DEEP_RESERVE = 128 items left unsealed past
# the head) and its items in flight per lane (RSF_DEEP_U = 8)
bash scripts/ab.sh abx 2 gossip default u1_16 u2_8 u2_32 res64 res256 du4 || exit 1
