"""CPU-only checks of the oracle's gossip world: the threaded round (the CPU
baseline's all-core rate) is identical to the sequential restatement."""
import ctypes as C

import numpy as np
import pytest

import gossip_harness as H
import oracle_ffi as O
from ruserf_amd import gossip as G
from ruserf_amd import workload as W

L = O.lib()


@pytest.mark.parametrize("kind", ["intents", "churn"])
def test_threaded_round_identical(kind):
    n, rounds = 3000, 10
    if kind == "intents":
        s = 40
        subj, acts, ml = W.intents_workload(n, s, rounds, rate=0.02, seed=5, prune_frac=0.3)
    else:
        subj, acts, ml = W.churn_workload(n, rounds, events_per_round=30, queries_per_round=5, seed=5)
        s = len(subj)
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=16, gossip_limit=300, max_rumors=1 << 15,
                         event_buffer_size=64, query_buffer_size=64, slot_k=4)
    views = W.initial_views(s)
    w1 = H.oracle_world(cfg, subj, views)
    w7 = H.oracle_world(cfg, subj, views)
    for t in range(rounds):
        H.oracle_round(w1, t, ml[t], acts[t], threads=1)
        H.oracle_round(w7, t, ml[t], acts[t], threads=7)
        H.assert_same(H.world_state(w7), H.world_state(w1), f"round {t}")
    assert w1.merges == w7.merges > 0 and w1.sends == w7.sends
    L.orc_world_free(C.byref(w1))
    L.orc_world_free(C.byref(w7))


def test_rumor_ring_wraps_and_expires():
    """A ring of 128 slots over 30 rounds: blocks restart at slot 0 with the next
    generation; two generations stay resident (by parity), so when the ring wraps the
    queued ids of generation gen - 2 expire; threaded and sequential rounds agree."""
    n, rounds = 800, 30
    subj, acts, ml = W.churn_workload(n, rounds, events_per_round=20, queries_per_round=3, seed=8)
    s = len(subj)
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=24, gossip_limit=300, max_rumors=128,
                         event_buffer_size=64, query_buffer_size=64, slot_k=8, max_refute=2)
    views = W.initial_views(s)
    w1 = H.oracle_world(cfg, subj, views)
    w4 = H.oracle_world(cfg, subj, views)
    for t in range(rounds):
        H.oracle_round(w1, t, ml[t], acts[t], threads=1)
        H.oracle_round(w4, t, ml[t], acts[t], threads=4)
    H.assert_same(H.world_state(w4), H.world_state(w1), "ring")
    assert w1.rbits == 7 and w1.gen >= 3
    live = [((w1.gen - k) << 7) | 5 for k in (0, 1)]
    stale_id = ((w1.gen - 2) << 7) | 5
    assert all(L.orc_rumor_live(C.byref(w1), i) == 1 for i in live)
    assert L.orc_rumor_live(C.byref(w1), stale_id) == 0
    # generation parity picks the table half
    assert L.orc_rumor_index(C.byref(w1), live[0]) != L.orc_rumor_index(C.byref(w1), live[1])
    assert O.arr(w1.q_expired, n, np.uint32).sum() > 0
    # every queued id is of a live generation
    q = O.arr(w1.q_rumor, n * 3 * cfg.queue_cap, np.uint32)
    assert all(L.orc_rumor_live(C.byref(w1), int(i)) for i in np.unique(q[q != 0xFFFFFFFF]))
    L.orc_world_free(C.byref(w1))
    L.orc_world_free(C.byref(w4))
