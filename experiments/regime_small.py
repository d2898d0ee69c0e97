"""Oracle-only calibration of a small-N twin of the bench's reference queue regime (depth
8704, staggered ticks every 150 rounds to 4096): which (n, rate, retransmit_mult) puts the
intent queues at the bench's occupancy (4-8.4k items) so the bit-exact regime test
exercises the same deferred-path classes and checker sizes.  CPU only (test infrastructure).

usage: python experiments/regime_small.py N RATE MULT ROUNDS [THREADS]"""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import gossip_harness as H  # noqa: E402
import oracle_ffi as O  # noqa: E402
from ruserf_amd import gossip as G  # noqa: E402
from ruserf_amd import workload as W  # noqa: E402

n, rate, mult, rounds = int(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
th = int(sys.argv[5]) if len(sys.argv) > 5 else 8
s, depth, period, mx = 4096, 8704, 150, 4096
per_round = s * 4 + max(1, int(round(n * rate)))
ring = 1 << max(10, (per_round * rounds - 1).bit_length())
cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=64, queue_depth=(depth, 0, 0), gossip_limit=8 * 24,
                     gossip_overhead=2, retransmit_mult=mult, max_rumors=ring, event_buffer_size=512,
                     query_buffer_size=512, slot_k=1)
subj, acts, ml = W.intents_workload(n, s, rounds, rate=rate, seed=0x5EED, prune_frac=0.1)
w = H.oracle_world(cfg, subj, W.initial_views(s))
H.L.orc_world_set_checker(C.byref(w), mx, 0, 128, period)
t0 = time.time()
for t in range(rounds):
    H.oracle_round(w, t, ml[t], acts[t], threads=th)
    if (t + 1) % 30 == 0 or t == rounds - 1:
        hw = H.world_width(w)
        q = O.arr(w.q_rumor, n * 3 * depth, np.uint32).reshape(n, 3, depth)[:, 0, :hw]
        ql = (q != 0xFFFFFFFF).sum(axis=1)
        print(f"round {t}: {time.time() - t0:.1f}s hwm {hw} q mean {ql.mean():.0f} p50 {np.median(ql):.0f} "
              f"p99 {np.percentile(ql, 99):.0f} max {ql.max()} pruned {int(O.arr(w.q_pruned, n, np.uint32).sum())} "
              f"chk {list(w.chk_stats)}", flush=True)
H.L.orc_world_free(C.byref(w))
