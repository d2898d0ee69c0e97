"""GPU parity of the gossip round (member-state merge + dissemination) against
the CPU oracle: bit-exact over clocks, views, queues, dedup rings, digests of
delivered events, refutations and error bits."""
import ctypes as C
import os

import numpy as np
import pytest

import gossip_harness as H
import oracle_ffi as O
from ruserf_amd import gossip as G
from ruserf_amd import workload as W

pytestmark = pytest.mark.gpu
L = O.lib()


def pair(cfg, subj_member, views):
    g = G.GossipEngine(cfg)
    g.set_subjects(subj_member)
    g.init_views(*views)
    w = H.oracle_world(cfg, subj_member, views)
    return g, w


@pytest.mark.parametrize("n,s,rounds,rate,qcap,limit", [
    (2000, 64, 12, 0.01, 64, 8 * 24),
    (1500, 100, 10, 0.03, 16, 8 * 24),
    (700, 50, 15, 0.02, 8, 1400),
    (3000, 32, 8, 0.005, 64, 3 * 24),
    (1000, 40, 8, 0.05, 64, 4000),  # 192 record slots per (sender, peer) group: groups span several chunks
])
def test_intent_rounds_bit_exact(n, s, rounds, rate, qcap, limit):
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=qcap, gossip_limit=limit, max_rumors=1 << 16,
                         event_buffer_size=64, query_buffer_size=64, slot_k=4)
    subj, acts, ml = W.intents_workload(n, s, rounds, rate=rate, seed=7 + n)
    views = W.initial_views(s)
    g, w = pair(cfg, subj, views)
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t])
        H.assert_same(H.engine_state(g), H.world_state(w), f"round {t}")
    assert w.merges > 0
    st = H.engine_state(g)
    assert int(np.sum(st["clock"])) > n  # clocks advanced
    # views start KNOWN: entries that are not were erased by a pruned force_leave
    assert np.any(st["v_kind"] != G.KIND_KNOWN)
    g.close()
    L.orc_world_free(C.byref(w))


@pytest.mark.parametrize("qcap", [64, 256])
def test_bench_shape_bit_exact(qcap):
    """The bench's configuration (4096 subjects, queue_cap 64, 8 intents of budget per
    target, slot_k 1, 512-slot dedup rings) at 20k members with 5% originating per round:
    the queues saturate as in the bench (every member receives far more new intents than
    it can send), so bounded-queue prunes, full pending lists and merge_big_kernel are all
    on the path; bit-exact against the oracle after every round.  queue_cap 256: the same
    saturated shape through the four-slot-per-lane queues (gossip_queue4.h), whose prune
    path and full pending lists are then compared as well."""
    n, s, rounds = 20000, 4096, 12
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=qcap, gossip_limit=8 * 24, gossip_overhead=2,
                         max_rumors=1 << 18, event_buffer_size=512, query_buffer_size=512, slot_k=1)
    subj, acts, ml = W.intents_workload(n, s, rounds, rate=0.05, seed=2024)
    views = W.initial_views(s)
    g, w = pair(cfg, subj, views)
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t])
        H.assert_same(H.engine_state(g), H.world_state(w), f"round {t}")
    st = H.engine_state(g)
    assert int(st["q_pruned"].sum()) > 0  # saturated: the bounded queues dropped items
    if qcap > 64:  # more than one slot per lane in use
        r = st["q_rumor"].reshape(n, 3, qcap)
        assert np.count_nonzero(r[:, 0, :] != 0xFFFFFFFF, axis=1).max() > 64
    g.close()
    L.orc_world_free(C.byref(w))


@pytest.mark.parametrize("qcap,limit,rate,n", [(256, 8 * 24, 0.05, 6000), (128, 4000, 0.05, 2000),
                                               (65, 1400, 0.03, 1500), (200, 6 * 24, 0.3, 800)])
def test_queue_cap_over_64_bit_exact(qcap, limit, rate, n):
    """Queues of 65..256 slots (four slots per lane of the emitting wave, gossip_queue4.h):
    queues filling past 64 items under the bench's 8-intent budget (qcap 256, 200), wide
    budgets that overflow a 128-slot queue (groups of up to 200 records), an odd capacity
    (65, overflowing); bit-exact against the oracle after every round, then two
    QueueChecker ticks."""
    s, rounds = 64, 12
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=qcap, gossip_limit=limit, gossip_overhead=2,
                         max_rumors=1 << 17, event_buffer_size=64, query_buffer_size=64, slot_k=4)
    subj, acts, ml = W.intents_workload(n, s, rounds, rate=rate, seed=qcap + n)
    g, w = pair(cfg, subj, W.initial_views(s))
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t])
        H.assert_same(H.engine_state(g), H.world_state(w), f"round {t}")
    r = g.queues()[0].reshape(n, 3, qcap)
    assert np.count_nonzero(r[:, 0, :] != 0xFFFFFFFF, axis=1).max() > 64  # more than one slot per lane in use
    for mx, mn, warn in [(4096, 0, 128), (100, 0, 64)]:
        got = g.check_queues(mx, mn, warn)
        exp = (C.c_uint64 * 9)()
        L.orc_check_queues(C.byref(w), mx, mn, warn, exp)
        assert list(got["queued"]) + list(got["warn"]) + list(got["pruned"]) == list(exp), (mx, mn, warn)
        H.assert_same(H.engine_state(g), H.world_state(w), f"checker {mx}")
    g.close()
    L.orc_world_free(C.byref(w))


def test_queue_cap_256_churn_flood_ring_bit_exact():
    """qcap 256 with user events, queries and churn, and a rumor ring small enough to wrap:
    the four-slot-per-lane expiry, the query / event queues and their pending lists."""
    n, rounds = 1200, 40
    subj, acts, ml = W.churn_workload(n, rounds, events_per_round=25, queries_per_round=4, seed=78)
    s = len(subj)
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=256, gossip_limit=600, max_rumors=256,
                         event_buffer_size=128, query_buffer_size=128, slot_k=8, max_refute=2)
    g, w = pair(cfg, subj, W.initial_views(s))
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t])
        H.assert_same(H.engine_state(g), H.world_state(w), f"round {t}")
    st = H.engine_state(g)
    assert w.gen >= 3 and st["q_expired"].sum() > 0
    g.close()
    L.orc_world_free(C.byref(w))


def test_rumor_ring_recycles_bit_exact():
    """A rumor ring far smaller than the run: blocks restart the ring with the next
    generation, two generations resident; at each wrap the queued ids of generation
    gen - 2 expire, identically to the oracle (churn + flood: intents, events, queries)."""
    n, rounds = 1200, 40
    subj, acts, ml = W.churn_workload(n, rounds, events_per_round=25, queries_per_round=4, seed=77)
    s = len(subj)
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=24, gossip_limit=300, max_rumors=256,
                         event_buffer_size=128, query_buffer_size=128, slot_k=8, max_refute=2)
    g, w = pair(cfg, subj, W.initial_views(s))
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t])
        H.assert_same(H.engine_state(g), H.world_state(w), f"round {t}")
    st = H.engine_state(g)
    assert w.gen >= 3 and st["q_expired"].sum() > 0
    g.close()
    L.orc_world_free(C.byref(w))


def test_long_run_ring_1m():
    """2,000 rounds at 1M members (configs[1] size) with the default-size ring: no
    RSF_ERR_OVERFLOW however long the engine runs; clocks keep advancing."""
    n, s, rounds = 1_000_000, 64, 2000
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=16, max_rumors=1 << 16, event_buffer_size=8,
                         query_buffer_size=8, slot_k=1, max_refute=1)
    subj, acts, ml = W.intents_workload(n, s, 50, rate=0.001, seed=3)
    g = G.GossipEngine(cfg)
    g.set_subjects(subj)
    g.init_views(*W.initial_views(s))
    c0 = None
    for t in range(rounds):
        g.round(t, ml[t % 50], acts[t % 50])
        if t == 10:
            c0 = g.members()["clock"].copy()
    m = g.members()
    assert np.all(m["clock"] >= c0) and m["clock"].max() > c0.max()
    assert int(g.expired().astype(np.uint64).sum()) >= 0
    g.close()


@pytest.mark.parametrize("prune_frac", [0.0, 0.5, 1.0])
def test_prune_and_queue_overflow_bit_exact(prune_frac):
    """force_leave(prune) -> handle_prune (base.rs:1587-1612) erases the member at every
    receiver that accepts the leave (Reap event), the next intent is buffered; small
    queues overflow, and every dropped live item is counted (q_pruned) and flagged
    (RSF_E_QUEUE_PRUNE) identically to the oracle.  Ends with a QueueChecker tick."""
    n, s, rounds = 1500, 24, 14
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=6, gossip_limit=4 * 24, max_rumors=1 << 16,
                         event_buffer_size=64, query_buffer_size=64, slot_k=4)
    subj, acts, ml = W.intents_workload(n, s, rounds, rate=0.03, seed=21, prune_frac=prune_frac)
    views = W.initial_views(s)
    g, w = pair(cfg, subj, views)
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t])
        H.assert_same(H.engine_state(g), H.world_state(w), f"round {t}")
    st = H.engine_state(g)
    assert st["q_pruned"].sum() > 0 and np.all((st["err"] & G.E_QUEUE_PRUNE != 0) == (st["q_pruned"] > 0))
    erased = np.count_nonzero(st["v_kind"] != G.KIND_KNOWN)
    assert (erased > 0) == (prune_frac > 0)
    for mx, mn, warn in [(4096, 0, 128), (3, 0, 2), (0, 2, 1)]:
        got = g.check_queues(mx, mn, warn)
        exp = (C.c_uint64 * 9)()
        L.orc_check_queues(C.byref(w), mx, mn, warn, exp)
        assert list(got["queued"]) + list(got["warn"]) + list(got["pruned"]) == list(exp), (mx, mn, warn)
        H.assert_same(H.engine_state(g), H.world_state(w), f"checker {mx}")
    g.close()
    L.orc_world_free(C.byref(w))


@pytest.mark.parametrize("n,rounds", [(3000, 14), (1200, 20)])
def test_churn_and_flood_bit_exact(n, rounds):
    cfg = G.GossipConfig(n_members=n, n_subjects=max(1, n // 100), queue_cap=32, gossip_limit=400,
                         max_rumors=1 << 16, event_buffer_size=512, query_buffer_size=512, slot_k=8)
    subj, acts, ml = W.churn_workload(n, rounds, events_per_round=30, queries_per_round=5, seed=11 + n)
    views = W.initial_views(len(subj))
    g, w = pair(cfg, subj, views)
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t])
        H.assert_same(H.engine_state(g), H.world_state(w), f"round {t}")
    st = H.engine_state(g)
    assert np.any(st["eb_cnt"] > 0) and np.any(st["qb_cnt"] > 0)
    assert np.any(st["v_status"] == G.STATUS_LEFT) or np.any(st["v_status"] == G.STATUS_FAILED)
    g.close()
    L.orc_world_free(C.byref(w))


@pytest.mark.parametrize("limits", [(512, 1024), (300, 1100)])
def test_churn_flood_oversized_originations_bit_exact(limits):
    """A churn flood where a fifth of the user events and queries have sizes around the
    entry points' limits (Serf::user_event, api.rs:255-287; query_in, base.rs:916-921):
    every action's status (ok / skipped / the SerfError) and the whole state after every
    round are bit-exact against the oracle; some actions of each kind are rejected and
    some large ones accepted (that a rejected action moves no clock is asserted directly by
    test_reference_kats_gpu.py's size-limit tests)."""
    ue, ql = limits
    n, rounds = 1500, 14
    cfg = G.GossipConfig(n_members=n, n_subjects=15, queue_cap=32, gossip_limit=1400, max_rumors=1 << 16,
                         event_buffer_size=512, query_buffer_size=512, slot_k=8, max_user_event_size=ue,
                         query_size_limit=ql)
    subj, acts, ml = W.churn_workload(n, rounds, events_per_round=30, queries_per_round=6, seed=ue + ql,
                                      oversize=0.2)
    g, w = pair(cfg, subj, W.initial_views(len(subj)))
    seen = set()
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t])
        got = g.action_status()
        exp = np.zeros(len(acts[t]), np.int32)
        if len(exp):
            assert L.orc_world_action_status(C.byref(w), exp.ctypes.data_as(C.POINTER(C.c_int32)), len(exp)) == 0
        assert np.array_equal(got, exp), f"round {t} action status"
        seen.update(int(x) for x in got)
        H.assert_same(H.engine_state(g), H.world_state(w), f"round {t}")
        a = acts[t]
        big = (a["act"] == G.ACT_USER_EVENT) & (a["payload_len"] > 32)
        seen.add(("big_ok", bool(np.any(big & (got == G.ACT_OK)))))
    assert {G.ERR_USER_EVENT_LIMIT, G.ERR_QUERY_TOO_LARGE, G.ACT_OK} <= seen, seen
    if ue >= 512:  # names 1..64 + payloads 420..560: some fit the default limit
        assert ("big_ok", True) in seen
    g.close()
    L.orc_world_free(C.byref(w))


def test_queue_checker_per_member_max_bit_exact():
    """QueueChecker with min_queue_depth > 0 (get_queue_max, base.rs:748-759): each
    member's max is 2 * its own members.states.len() -- the untracked members, itself and
    the subjects it knows -- so members that know different numbers of subjects prune at
    different depths.  Most members are subjects and start unknown; a random share of the
    (member, subject) entries is set known, differently per member.  Bit-exact against the
    oracle (counts and state), then a round on, and again."""
    n, s, rounds = 80, 76, 10
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=64, gossip_limit=1400, max_rumors=1 << 14,
                         event_buffer_size=64, query_buffer_size=64, slot_k=4)
    subj, acts, ml = W.intents_workload(n, s, rounds + 2, rate=0.1, seed=31, prune_frac=0.0)
    views = (np.zeros(s, np.uint8), np.zeros(s, np.uint8), np.zeros(s, np.uint64))
    g, w = pair(cfg, subj, views)
    rng = np.random.default_rng(5)
    vk = O.arr(w.v_kind, n * s, np.uint8).reshape(n, s)
    vs = O.arr(w.v_status, n * s, np.uint8).reshape(n, s)
    for m in range(n):
        for j in rng.choice(s, size=int(rng.integers(0, 20)), replace=False):
            g.set_view(m, int(j), G.KIND_KNOWN, G.STATUS_ALIVE, 0)
            vk[m, j], vs[m, j] = G.KIND_KNOWN, G.STATUS_ALIVE
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t])
    H.assert_same(H.engine_state(g), H.world_state(w), "before the checker")
    total_pruned = 0
    for k, (mx, mn, warn) in enumerate([(4096, 1, 8), (4096, 30, 8)]):
        got = g.check_queues(mx, mn, warn)
        exp = (C.c_uint64 * 9)()
        L.orc_check_queues(C.byref(w), mx, mn, warn, exp)
        assert list(got["queued"]) + list(got["warn"]) + list(got["pruned"]) == list(exp), (mx, mn, warn)
        total_pruned += sum(got["pruned"])
        H.assert_same(H.engine_state(g), H.world_state(w), f"checker {mn}")
        g.round(rounds + k, ml[rounds + k], acts[rounds + k])
        H.oracle_round(w, rounds + k, ml[rounds + k], acts[rounds + k])
        H.assert_same(H.engine_state(g), H.world_state(w), f"round after checker {mn}")
    assert total_pruned > 0
    g.close()
    L.orc_world_free(C.byref(w))


def test_queues_width_on_plain_queues():
    """GossipEngine.queues(width) on a context without deep queues (queue_depth None):
    the first `width` items of every queue, equal to the plain dump truncated, and
    max_live = the most items any queue holds."""
    n, s, rounds = 600, 32, 6
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=16, max_rumors=1 << 15, event_buffer_size=32,
                         query_buffer_size=32, slot_k=2)
    subj, acts, ml = W.intents_workload(n, s, rounds, rate=0.05, seed=3)
    g = G.GossipEngine(cfg)
    g.set_subjects(subj)
    g.init_views(*W.initial_views(s))
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
    full = [np.asarray(x) for x in g.queues()]
    for width in (4, 16, 20):
        part = [np.asarray(x) for x in g.queues(width=width)]
        w = min(width, 16)
        live3 = full[0].reshape(n, 3, 16)[:, :, :w] != 0xFFFFFFFF  # free slots' other fields are unspecified
        for idx, (a, b) in enumerate(zip(full[:4], part[:4])):
            a3, b3 = a.reshape(n, 3, 16)[:, :, :w], b.reshape(n, 3, width)
            assert np.array_equal(np.where(live3, a3, 0), np.where(live3, b3[:, :, :w], 0)), idx
            if width > 16:
                assert np.all(b3[:, :, 16:] == (0xFFFFFFFF if idx == 0 else 0))
        assert np.array_equal(live3, part[0].reshape(n, 3, width)[:, :, :w] != 0xFFFFFFFF)
        assert np.array_equal(full[4], part[4])
        live = np.count_nonzero(full[0].reshape(n * 3, 16) != 0xFFFFFFFF, axis=1).max()
        assert g.max_live == live
    g.close()


def test_unknown_subjects_buffer_intents_then_join():
    """Subjects start unknown: intents go to the recent-intent buffer
    (upsert_intent), and a memberlist NotifyJoin consumes it (handle_node_join)."""
    n, s, rounds = 800, 20, 10
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=32, max_rumors=1 << 15,
                         event_buffer_size=32, query_buffer_size=32, slot_k=2)
    # no pruned force_leaves here: a prune after the NotifyJoin would erase the member again
    subj, acts, _ = W.intents_workload(n, s, rounds, rate=0.02, seed=99, prune_frac=0.0)
    views = (np.zeros(s, np.uint8), np.zeros(s, np.uint8), np.zeros(s, np.uint64))
    g, w = pair(cfg, subj, views)
    for t in range(rounds):
        ml = np.zeros(0, G.ML_DTYPE)
        if t == 6:
            ml = np.zeros(s, G.ML_DTYPE)
            ml["subject"] = np.arange(s)
            ml["kind"] = G.ML_JOIN
            ml["set_alive"] = 2
        g.round(t, ml, acts[t])
        H.oracle_round(w, t, ml, acts[t])
        H.assert_same(H.engine_state(g), H.world_state(w), f"round {t}")
    kinds = H.engine_state(g)["v_kind"].copy()
    # a subject does not receive memberlist's NotifyJoin about itself (m == subject is skipped)
    kinds[subj, np.arange(s)] = G.KIND_KNOWN
    assert np.all(kinds == G.KIND_KNOWN)
    g.close()
    L.orc_world_free(C.byref(w))


def test_apply_batch_matches_oracle_handlers():
    """notify_message over a random batch (join/leave intents, user events,
    queries), several messages per receiver, in array order per receiver."""
    n, s = 300, 12
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=8, max_rumors=1024, event_buffer_size=16,
                         query_buffer_size=16, slot_k=4)
    subj = W.subjects_for(n, s)
    rng = np.random.default_rng(5)
    kinds = rng.integers(0, 4, s).astype(np.uint8)
    status = rng.integers(0, 5, s).astype(np.uint8)
    lt = rng.integers(0, 20, s).astype(np.uint64)
    g, w = pair(cfg, subj, (kinds, status, lt))
    for rep in range(4):
        k = 3000
        msgs = np.zeros(k, G.MSG_DTYPE)
        msgs["receiver"] = rng.integers(0, n, k)
        msgs["type"] = rng.choice([G.MSG_JOIN, G.MSG_LEAVE, G.MSG_USER_EVENT, G.MSG_QUERY], k)
        msgs["subject"] = rng.integers(0, s, k)
        msgs["ltime"] = rng.integers(0, 60 + 40 * rep, k)
        msgs["key"] = rng.integers(0, 6, k)
        msgs["flags"] = rng.integers(0, 2, k)
        flags, refute = g.apply_batch(msgs)
        for i in range(k):
            m, t = int(msgs["receiver"][i]), int(msgs["type"][i])
            ref = C.c_uint64(0)
            if t == G.MSG_JOIN:
                f = L.orc_handle_join_intent(C.byref(w), m, int(msgs["subject"][i]), int(msgs["ltime"][i]))
            elif t == G.MSG_LEAVE:
                f = L.orc_handle_leave_intent(C.byref(w), m, int(msgs["subject"][i]), int(msgs["ltime"][i]),
                                              int(msgs["flags"][i]), C.byref(ref))
            elif t == G.MSG_USER_EVENT:
                f = L.orc_handle_user_event(C.byref(w), m, int(msgs["ltime"][i]), int(msgs["key"][i]))
            else:
                f = L.orc_handle_query(C.byref(w), m, int(msgs["ltime"][i]), int(msgs["key"][i]), int(msgs["flags"][i]))
            assert flags[i] == f, (rep, i, t)
            if f & O.F_REFUTE:
                assert refute[i] == ref.value
        H.assert_same(H.engine_state(g), H.world_state(w), f"batch {rep}")
    g.close()
    L.orc_world_free(C.byref(w))


def test_large_round_properties():
    """1M members (BASELINE configs[1] size), 256 subjects: invariants that hold at
    any size — Lamport clocks never decrease and exceed every status_time a
    member has accepted, queue transmit counts stay under the retransmit limit,
    and two runs with the same seed are identical."""
    n, s, rounds = 1_000_000, 256, 4
    cfg = G.GossipConfig(n_members=n, n_subjects=s, max_rumors=1 << 20, event_buffer_size=8, query_buffer_size=8,
                         slot_k=1)
    subj, acts, ml = W.intents_workload(n, s, rounds, rate=0.01, seed=1)
    digests = []
    for rep in range(2):
        g = G.GossipEngine(cfg)
        g.set_subjects(subj)
        g.init_views(*W.initial_views(s))
        prev = None
        for t in range(rounds):
            g.round(t, ml[t], acts[t])
            m = g.members()
            if prev is not None:
                assert np.all(m["clock"] >= prev)
            prev = m["clock"]
        lt, st, kd = g.view()
        lt = lt.reshape(n, s)
        known = kd.reshape(n, s) == G.KIND_KNOWN
        # every status_time accepted from a message was witnessed: clock > ltime (initial views hold ltime 1)
        accepted = np.where(known & (lt > 1), lt, 0).max(axis=1)
        assert np.all(accepted < prev)
        r, sq, tx, ln, ns = g.queues()
        limit = O.lib().orc_retransmit_limit(4, n)
        assert np.all(tx[r != 0xFFFFFFFF] < limit)
        sent, merged = g.last_round_stats()
        assert sent > 0 and merged == sent
        digests.append((m["digest"].copy(), lt.sum()))
        g.close()
    assert np.array_equal(digests[0][0], digests[1][0]) and digests[0][1] == digests[1][1]


def test_configs1_full_shape_properties():
    """BASELINE configs[1] as specified: 1M members, 4096 tracked subjects, 32 rounds of
    the 1% intent workload (prune mix included).  The view (64 GB) is too large for the
    oracle, so size-independent properties: clocks never decrease; on sampled rows every
    accepted status_time was witnessed (clock > ltime); transmits stay under the limit;
    no capacity error but the counted queue prunes; the same seed gives the same
    digests and sampled views."""
    n, s, rounds = 1_000_000, 4096, 32
    cfg = G.GossipConfig(n_members=n, n_subjects=s, max_rumors=1 << 20, event_buffer_size=8, query_buffer_size=8,
                         slot_k=1)
    subj, acts, ml = W.intents_workload(n, s, rounds, rate=0.01, seed=3, prune_frac=0.1)
    sample = [(0, 64), (n // 2 - 32, 64), (n - 64, 64)]
    runs = []
    for rep in range(2):
        g = G.GossipEngine(cfg)
        g.set_subjects(subj)
        g.init_views(*W.initial_views(s))
        prev = None
        for t in range(rounds):
            g.round(t, ml[t], acts[t])
            if t % 8 == 7 or t == rounds - 1:
                m = g.members()
                if prev is not None:
                    assert np.all(m["clock"] >= prev), t
                prev = m["clock"]
        assert np.all((m["err"] & ~np.uint32(G.E_QUEUE_PRUNE)) == 0)
        views = []
        for r0, cnt in sample:
            lt, st, kd = g.view(rows=(r0, cnt))
            lt, known = lt.reshape(cnt, s), kd.reshape(cnt, s) == G.KIND_KNOWN
            accepted = np.where(known & (lt > 1), lt, 0).max(axis=1)
            assert np.all(accepted < m["clock"][r0:r0 + cnt])
            views.append((lt.copy(), st.copy(), kd.copy()))
        r, sq, tx, ln, ns = g.queues()
        limit = O.lib().orc_retransmit_limit(4, n)
        assert np.all(tx[r != 0xFFFFFFFF] < limit)
        sent, merged = g.last_round_stats()
        assert sent > 0 and merged == sent
        assert all(g.cub_canaries())  # no hipCUB call wrote past its temporary storage
        runs.append((m["digest"].copy(), m["clock"].copy(), views))
        g.close()
    assert np.array_equal(runs[0][0], runs[1][0]) and np.array_equal(runs[0][1], runs[1][1])
    for a, b in zip(runs[0][2], runs[1][2]):
        for x, y in zip(a, b):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("runs", [False, True, "with_empty_runs", "buckets"])
def test_two_shards_equal_one_context(runs):
    """The multi-GPU split (round_begin / rumor-block sum / round_emit /
    all-to-all / round_merge or round_merge_runs) with two shard contexts on one
    GPU and the exchange done by hand must reproduce the single-context round
    exactly."""
    import torch
    from ruserf_amd.dist import hbm_tensor
    n, rounds = 4000, 10
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    subj, acts, ml = W.churn_workload(n, rounds, events_per_round=20, queries_per_round=4, seed=3)
    s = len(subj)
    base = dict(n_members=n, n_subjects=s, queue_cap=32, max_rumors=1 << 16, event_buffer_size=128,
                query_buffer_size=128, slot_k=8)
    views = W.initial_views(s)
    one = G.GossipEngine(G.GossipConfig(**base))
    one.set_stream(stream.cuda_stream)
    shards = [G.GossipEngine(G.GossipConfig(**base, shard=(0, n // 2))),
              G.GossipEngine(G.GossipConfig(**base, shard=(n // 2, n)))]
    for e in [one] + shards:
        e.set_stream(stream.cuda_stream)
        e.set_subjects(subj)
        e.init_views(*views)
    for t in range(rounds):
        one.round(t, ml[t], acts[t])
        for e in shards:
            e.round_begin(t, ml[t], acts[t])
        blocks = [hbm_tensor(*e.rumor_block()[:1], e.rumor_block()[1] // 8) for e in shards]
        total = blocks[0] + blocks[1]
        for b in blocks:
            b.copy_(total)
        if runs == "buckets":  # fixed-capacity buckets, the all-to-all done by hand
            bufs = [e.bucket_buffers(2) for e in shards]
            words = bufs[0][2] // 4
            for e in shards:
                e.round_emit_buckets(2)
            stream.synchronize()
            for dst, e in enumerate(shards):
                recv = hbm_tensor(bufs[dst][1], 2 * words, "<i4")
                for src in range(2):
                    send = hbm_tensor(bufs[src][0], 2 * words, "<i4")
                    recv[src * words:(src + 1) * words].copy_(send[dst * words:(dst + 1) * words])
            stream.synchronize()
            for e in shards:
                e.round_merge_buckets(2)
            stream.synchronize()
            assert all(e.bucket_ok() for e in shards)
            full = H.normalize_queues(H.engine_state(one))
            halves = [H.normalize_queues(H.engine_state(e)) for e in shards]
            for k in full:
                assert np.array_equal(np.concatenate([halves[0][k], halves[1][k]]), full[k]), (t, k)
            continue
        counts = [e.round_emit(2) for e in shards]
        sends = [hbm_tensor(e.send_buffer()[0], int(c.sum())) for e, c in zip(shards, counts)]
        for dst, e in enumerate(shards):
            parts = []
            for src in range(2):
                off = int(counts[src][:dst].sum())
                parts.append(sends[src][off: off + int(counts[src][dst])])
            recv = torch.cat(parts).contiguous()
            if runs:
                counts_r = [p.numel() for p in parts]
                if runs == "with_empty_runs":  # sources that sent nothing change nothing
                    counts_r = [0] + counts_r[:1] + [0, 0] + counts_r[1:] + [0]
                e.round_merge_runs(recv.data_ptr(), counts_r)
                assert e.runs_ok()
            else:
                e.round_merge(recv.data_ptr(), recv.numel())
            stream.synchronize()
        torch.cuda.synchronize()
        full = H.normalize_queues(H.engine_state(one))
        halves = [H.normalize_queues(H.engine_state(e)) for e in shards]
        for k in full:
            got = np.concatenate([halves[0][k], halves[1][k]])
            assert np.array_equal(got, full[k]), (t, k)
    for e in [one] + shards:
        e.close()


def _threads():
    import os
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", n)), 16))


def _oracle_deliveries(w):
    """the oracle's delivery log as (member, ltime, key, cc, kind) rows, member-major (a member
    event's flags word holds LOG_MEMBER: kind 1, its ltime word = the type)"""
    n, cap = w.n, w.dcap
    cnt = np.minimum(O.arr(w.dcnt, n, np.uint32), cap)
    log = O.arr(w.dlog, n * cap * 3, np.uint64).reshape(n, cap, 3)
    mask = np.arange(cap)[None, :] < cnt[:, None]
    mem = np.broadcast_to(np.arange(n, dtype=np.uint32)[:, None], (n, cap))[mask]
    e = log[mask]
    kind = ((e[:, 2] & np.uint64(O.LOG_MEMBER)) != 0).astype(np.uint8)
    cc = (e[:, 2] & np.uint64(O.LOG_CC)).astype(np.uint8)
    return mem, e[:, 0], e[:, 1], cc, kind


def test_configs3_100k_churn_flood_coalesce():
    """BASELINE configs[3] at full size: 100k members, 1% churn (1000 subjects fail or
    leave, a quarter of the failures force-left with prune), a flood of 100 user events
    (16 names, 32-B payloads, cc 50%) + 10 queries per round, event/query buffers 512,
    retransmit mult 4.  Bit-exact against the oracle every round (clocks, digests of
    every delivery, error bits, queue drops, the delivery log of user and member events);
    the full state at the end.  Each member's member events go through the GPU
    MemberEventCoalescer (coalesce/member.rs:60-118), one per member, a quantum per round,
    bit-exact against the oracle's; each member's cc deliveries then go through the GPU
    UserEventCoalescer (coalesce/user.rs:52-97), checked against the oracle's coalescer on
    a sample of members."""
    from ruserf_amd.coalesce import MEMBER_EVENT_DTYPE, NO_EVENT, USER_EVENT_DTYPE, MemberEventCoalescer, \
        coalesce_user_events
    n, rounds = 100_000, 9
    subj, acts, ml = W.churn_workload(n, rounds, events_per_round=100, queries_per_round=10, seed=2024)
    s = len(subj)
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=64, gossip_limit=1400, max_rumors=1 << 16,
                         event_buffer_size=512, query_buffer_size=512, slot_k=16)
    g, w = pair(cfg, subj, W.initial_views(s))
    dcap = 512
    g.set_delivery_log(dcap)
    assert L.orc_world_set_delivery_log(C.byref(w), dcap) == 0
    th = _threads()
    logs = []
    mcoal = MemberEventCoalescer(n, s)
    mlast = np.full((n, s), NO_EVENT, np.uint8)
    n_mev = n_mflushed = 0
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t], threads=th)
        m = g.members()
        for k, ok in [("clock", w.clock), ("event_clock", w.eclock), ("query_clock", w.qclock),
                      ("digest", w.digest), ("err", w.err)]:
            exp = O.arr(ok, n, np.uint32 if k == "err" else np.uint64)
            assert np.array_equal(m[k], exp), (t, k)
        assert np.array_equal(g.pruned(), O.arr(w.q_pruned, n, np.uint32)), t
        d = g.deliveries()
        om, ol, ok_, oc, okind = _oracle_deliveries(w)
        assert np.array_equal(d["member"], om) and np.array_equal(d["ltime"], ol), t
        assert np.array_equal(d["key"], ok_) and np.array_equal(d["cc"], oc), t
        assert np.array_equal(d["kind"], okind), t
        me = d[d["kind"] == G.DELIVERY_MEMBER_EVENT]
        mev = np.zeros(len(me), MEMBER_EVENT_DTYPE)
        mev["group"], mev["node"], mev["type"] = me["member"], me["key"], me["ltime"]
        got_m = mcoal.flush(mev)
        assert np.array_equal(got_m, O.member_coalesce(mlast, mev)), t
        n_mev += len(mev)
        n_mflushed += len(got_m)
        logs.append(d[d["kind"] == G.DELIVERY_USER_EVENT])
    H.assert_same(H.engine_state(g), H.world_state(w), "final")
    st = H.engine_state(g)
    assert np.any(st["v_status"] == G.STATUS_LEFT) and np.any(st["v_kind"] == G.KIND_UNKNOWN)
    assert 0 < n_mflushed < n_mev  # member events were produced and some coalesced away
    assert np.array_equal(mcoal.last_events(), mlast)
    mcoal.close()
    # coalescing of the cc deliveries, one coalescer per member (stable by member: arrival order kept)
    d = np.concatenate(logs)
    d = d[d["cc"] == 1]
    order = np.argsort(d["member"], kind="stable")
    d = d[order]
    ev = np.zeros(len(d), USER_EVENT_DTYPE)
    ev["group"] = d["member"]
    ev["name"] = (d["key"] >> np.uint64(32)).astype(np.uint32)
    ev["ltime"] = d["ltime"]
    ev["payload"] = d["key"] & np.uint64(0xFFFFFFFF)
    got = coalesce_user_events(ev)
    assert 0 < len(got) < len(ev)
    sample = np.random.default_rng(1).choice(np.unique(ev["group"]), 2000, replace=False)
    bounds = np.searchsorted(ev["group"], np.stack([sample, sample + 1]))
    gb = np.searchsorted(got["group"], np.stack([sample, sample + 1]))
    for i in range(len(sample)):
        sel = ev[bounds[0, i]:bounds[1, i]]
        arr = (O.UEvent * len(sel))()
        for j, e in enumerate(sel):
            arr[j].name, arr[j].ltime, arr[j].payload = int(e["name"]), int(e["ltime"]), int(e["payload"])
        res = (O.UEvent * len(sel))()
        k = L.orc_coalesce_user_events(arr, len(sel), res)
        mine = got[gb[0, i]:gb[1, i]]
        assert k == len(mine)
        assert [(r.name, r.ltime, r.payload) for r in res[:k]] == \
            [(int(x["name"]), int(x["ltime"]), int(x["payload"])) for x in mine]
    g.close()
    L.orc_world_free(C.byref(w))


@pytest.mark.parametrize("qcap,fanout,mult,limit", [(64, 1, 1, 300), (64, 5, 2, 240), (64, 3, 1, 90),
                                                    (256, 4, 1, 260), (100, 2, 3, 500)])
def test_emission_pick_paths_bit_exact(qcap, fanout, mult, limit):
    """The queue-major emission (every peer's picks from one queue in a pass, q_pick_peers /
    q4_pick_peers) on the paths the bench shape rarely takes: one and five peers; a
    retransmit limit of 1-3 (every pick of a class retires, or classes run out within one
    emission and the exact per-peer fallback takes over); budgets that leave room for later
    shorter items (user events and queries of many lengths: skips break the prefix run);
    bit-exact against the oracle's per-peer broadcast_messages after every round."""
    n, rounds = 1500, 14
    subj, acts, ml = W.churn_workload(n, rounds, events_per_round=40, queries_per_round=6, seed=qcap * 7 + fanout)
    s = len(subj)
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=qcap, gossip_limit=limit, gossip_overhead=3,
                         fanout=fanout, retransmit_mult=mult, max_rumors=1 << 14, event_buffer_size=128,
                         query_buffer_size=128, slot_k=8)
    g, w = pair(cfg, subj, W.initial_views(s))
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t])
        H.assert_same(H.engine_state(g), H.world_state(w), f"round {t}")
    assert w.merges > 0
    g.close()
    L.orc_world_free(C.byref(w))
