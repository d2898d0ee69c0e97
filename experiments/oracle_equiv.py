"""Equivalence check of two oracle builds (round 6: the faster queue scans): runs the churn-flood
and regime workloads on the oracle and saves every world field; run once with OLD=<path of the
previous liboracle.so> and once without, then compare the two .npz files field by field.
CPU only (test infrastructure).  usage: [OLD=lib.so] python experiments/oracle_equiv.py OUT.npz"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, "/root/repo/tests")
sys.path.insert(0, "/root/repo")
import oracle_ffi as O  # noqa: E402

if os.environ.get("OLD"):
    O.LIB_PATH = os.environ["OLD"]
import gossip_harness as H  # noqa: E402
from ruserf_amd import gossip as G  # noqa: E402
from ruserf_amd import workload as W  # noqa: E402

out = sys.argv[1]
res = {}
# churn flood, small deep queues that fill, ring wraps, ticks
for qcap, depth, limit, mult in [(16, 100, 400, 4), (8, 40, 600, 2), (64, 200, 260, 1)]:
    n, rounds = 1200, 30
    subj, acts, ml = W.churn_workload(n, rounds, events_per_round=30, queries_per_round=5, seed=depth + qcap)
    s = len(subj)
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=qcap, queue_depth=(depth, depth, depth),
                         gossip_limit=limit, gossip_overhead=3, retransmit_mult=mult, max_rumors=512,
                         event_buffer_size=128, query_buffer_size=128, slot_k=8, max_refute=2)
    w = H.oracle_world(cfg, subj, W.initial_views(s))
    H.L.orc_world_set_checker(C.byref(w), depth // 3, 0, 8, 4)
    for t in range(rounds):
        H.oracle_round(w, t, ml[t], acts[t], threads=4)
        if t in (9, 19):
            exp = (C.c_uint64 * 9)()
            H.L.orc_check_queues(C.byref(w), depth // 2, 0, 8, exp)
    st = H.world_state(w)
    for k, v in st.items():
        res[f"{qcap}_{depth}_{k}"] = np.array(v)
    H.L.orc_world_free(C.byref(w))
# the regime shape, short
n, s, rounds = 5000, 4096, 90
cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=64, queue_depth=(8704, 0, 0), gossip_limit=8 * 24,
                     gossip_overhead=2, max_rumors=1 << 20, event_buffer_size=512, query_buffer_size=512, slot_k=1)
subj, acts, ml = W.intents_workload(n, s, rounds, rate=0.05, seed=77)
w = H.oracle_world(cfg, subj, W.initial_views(s))
H.L.orc_world_set_checker(C.byref(w), 900, 0, 128, 30)
for t in range(rounds):
    H.oracle_round(w, t, ml[t], acts[t], threads=8)
st = H.world_state(w, width=H.world_width(w))
for k, v in st.items():
    res[f"regime_{k}"] = np.array(v)
res["chk"] = np.array(list(w.chk_stats))
np.savez(out, **res)
print("done", H.world_width(w))
