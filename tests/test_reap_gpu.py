"""Reaper ticks (core/src/serf/base.rs:519-601, 1782-1784) on the GPU against the
oracle, bit for bit, inside a churn + flood run: failed and left members age out
by reconnect / tombstone timeout with Reap member events (digest), buffered
intents by recent_intent_timeout, and the rounds after the reaps keep matching.
The oracle's reaper is pinned by the reference's serf_reap_handler KAT
(tests/test_oracle_kat.py)."""
import ctypes as C

import numpy as np
import pytest

import gossip_harness as H
import oracle_ffi as O
from ruserf_amd import gossip as G
from ruserf_amd import workload as W

pytestmark = pytest.mark.gpu
L = O.lib()


@pytest.mark.parametrize("n,rounds,timeouts", [(1500, 18, (4, 6, 3)), (2500, 14, (2, 3, 2))])
def test_reap_ticks_bit_exact(n, rounds, timeouts):
    subj, acts, ml = W.churn_workload(n, rounds, churn=1.0 / 60, events_per_round=20, queries_per_round=2,
                                      seed=77 + n)
    cfg = G.GossipConfig(n_members=n, n_subjects=len(subj), queue_cap=32, gossip_limit=400,
                         max_rumors=1 << 16, event_buffer_size=128, query_buffer_size=128, slot_k=4)
    views = W.initial_views(len(subj))
    g = G.GossipEngine(cfg)
    g.set_subjects(subj)
    g.init_views(*views)
    w = H.oracle_world(cfg, subj, views)
    reconnect, tombstone, intent = timeouts
    reaped_any = False
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t])
        if t % 3 == 2:
            before = H.engine_state(g)
            g.reap(t, reconnect, tombstone, intent)
            assert L.orc_reap(C.byref(w), t, reconnect, tombstone, intent) == 0
            after = H.engine_state(g)
            reaped_any |= bool(np.any(before["v_kind"] != after["v_kind"]))
        H.assert_same(H.engine_state(g), H.world_state(w), f"round {t}")
    assert reaped_any
    g.close()
    L.orc_world_free(C.byref(w))
