"""Deep transmit-limited queues (queue_depth > queue_cap): a register head plus an unordered
HBM tail per queue, so a queue holds up to the reference's max_queue_depth (4096,
core/src/options.rs:512) and is pruned only by the QueueChecker (base.rs:720-760).  Bit-exact
against the oracle's bounded queue of the same depth (oracle/oracle.c orc_queue_insert /
orc_queue_get_broadcasts / orc_check_queues): emission decided from the head alone, the
members whose picks need the tail (emit_deep_wave_kernel), spills, the bounded prune at the full
depth, ring expiry of tail items, QueueChecker ticks, and the multi-GPU bucket emission."""
import ctypes as C

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


def same(g, w, ctx):
    e, o = H.deep_states(g, w)
    H.assert_same(e, o, ctx)


def check_both(g, w, mx, mn, warn, ctx):
    got = g.check_queues(mx, mn, warn)
    exp = (C.c_uint64 * 9)()
    L.orc_check_queues(C.byref(w), mx, mn, warn, exp)
    assert list(got["queued"]) + list(got["warn"]) + list(got["pruned"]) == list(exp), (ctx, mx, mn, warn)
    same(g, w, f"{ctx} checker {mx}")


@pytest.mark.parametrize("rounds", [12])
def test_deep_bench_shape_bit_exact(rounds):
    """The bench's saturated shape (20k members, 4096 subjects, 5% originating, 8 intents of
    budget per target) with the intent queue 4096 deep: nothing is dropped between checker
    ticks (the queues grow past the 64-slot head), and the state is bit-exact after every
    round; then a QueueChecker tick at max_queue_depth 128 prunes head and tail together."""
    n, s = 20000, 4096
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=64, queue_depth=(4096, 0, 0), gossip_limit=8 * 24,
                         gossip_overhead=2, max_rumors=1 << 18, event_buffer_size=512, query_buffer_size=512,
                         slot_k=1)
    subj, acts, ml = W.intents_workload(n, s, rounds, rate=0.05, seed=2024)
    g, w = pair(cfg, subj, W.initial_views(s))
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t], threads=16)
        same(g, w, f"round {t}")
    st = H.engine_state(g, H.world_width(w))
    assert int(st["q_pruned"].sum()) == 0  # nothing dropped between ticks
    assert H.world_width(w) > 64  # the queues hold more than the head
    total, _ = g.deep_stats()
    assert total > 0  # some emissions needed the tail
    check_both(g, w, 128, 0, 64, "bench shape")
    g.close()
    L.orc_world_free(C.byref(w))


def test_deep_steady_state_ticks_bit_exact():
    """The reference's queue regime over many rounds at the bench's saturated shape (4096
    subjects, 8 intents of budget per target, 5% originating; 8k members): the intent queue
    8192 deep grows ~24 items a round, QueueChecker ticks every 25 rounds prune it to 1 100
    (the second and third ticks prune), and the ring is sized so nothing expires.
    The deferred path runs its recent mode (the tail's sealed prefix stays in HBM), re-lists
    members whose recent part cannot decide, and the full-depth class -- every one of them
    bit-exact against the oracle, compared every 5 rounds and after every tick."""
    n, s, rounds, every, mx = 8000, 4096, 80, 25, 1100
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=64, queue_depth=(8192, 0, 0), gossip_limit=8 * 24,
                         gossip_overhead=2, max_rumors=1 << 20, event_buffer_size=512, query_buffer_size=512,
                         slot_k=1)
    subj, acts, ml = W.intents_workload(n, s, rounds, rate=0.05, seed=77)
    g, w = pair(cfg, subj, W.initial_views(s))
    pruned_at_ticks = 0
    cls0 = g.deep_class_stats()
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t], threads=16)
        if (t + 1) % 5 == 0:
            same(g, w, f"round {t}")
        if (t + 1) % every == 0:
            got = g.check_queues(mx, 0, 128)
            exp = (C.c_uint64 * 9)()
            L.orc_check_queues(C.byref(w), mx, 0, 128, exp)
            assert list(got["queued"]) + list(got["warn"]) + list(got["pruned"]) == list(exp), t
            pruned_at_ticks += int(got["pruned"][0])
            same(g, w, f"tick after round {t}")
    st = H.engine_state(g, H.world_width(w))
    assert int(st["q_pruned"].sum()) == 0  # nothing dropped between ticks
    assert int(st["q_expired"].sum()) == 0  # the ring never wrapped onto a queued item
    assert pruned_at_ticks > 0
    cls = g.deep_class_stats() - cls0
    assert cls[0] > 0 and cls[3] > 0, cls  # the recent mode's smallest class and the full depth both ran
    g.close()
    L.orc_world_free(C.byref(w))


def test_deep_staggered_ticks_bit_exact():
    """Staggered QueueChecker ticks (rsf_gossip_check_queues_phase: each node's checker on
    its own timer, one phase of 25 after every round) in the reference's queue regime at the
    bench's saturated shape: every member's intent queue is pruned to 1 100 once per 25
    rounds, at its own round, by the streaming prune; bit-exact against the oracle's phased
    tick (orc_check_queues_phase), compared every 5 rounds, and the accumulated counts equal."""
    n, s, rounds, period, mx = 8000, 4096, 80, 25, 1100
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=64, queue_depth=(8192, 0, 0), gossip_limit=8 * 24,
                         gossip_overhead=2, max_rumors=1 << 20, event_buffer_size=512, query_buffer_size=512,
                         slot_k=1)
    subj, acts, ml = W.intents_workload(n, s, rounds, rate=0.05, seed=78)
    g, w = pair(cfg, subj, W.initial_views(s))
    exp_tot = np.zeros(9, dtype=np.uint64)
    g.checker_stats(reset=True)
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t], threads=16)
        g.check_queues_phase(period, (t + 1) % period, mx, 0, 128)
        exp = (C.c_uint64 * 9)()
        L.orc_check_queues_phase(C.byref(w), mx, 0, 128, period, (t + 1) % period, exp)
        exp_tot += np.array(list(exp), dtype=np.uint64)
        if (t + 1) % 5 == 0:
            same(g, w, f"round {t}")
    got = g.checker_stats(reset=True)
    assert list(got["queued"]) + list(got["warn"]) + list(got["pruned"]) == list(exp_tot)
    assert int(exp_tot[6]) > 0
    assert list(g.checker_stats()["queued"]) == [0, 0, 0]  # reset
    st = H.engine_state(g, H.world_width(w))
    assert int(st["q_pruned"].sum()) == 0 and int(st["q_expired"].sum()) == 0
    g.close()
    L.orc_world_free(C.byref(w))


def test_deep_in_round_checker_bit_exact():
    """In-round staggered ticks (rsf_gossip_set_checker: every round r ticks the members with
    id = r mod 25 between its emission and its merge, on a second stream beside the merge)
    in the reference's queue regime at the bench's saturated shape; bit-exact against the
    oracle's tick at the same point (orc_world_set_checker), compared every 5 rounds, the
    accumulated counts equal."""
    n, s, rounds, period, mx = 8000, 4096, 80, 25, 1100
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=64, queue_depth=(8192, 0, 0), gossip_limit=8 * 24,
                         gossip_overhead=2, max_rumors=1 << 20, event_buffer_size=512, query_buffer_size=512,
                         slot_k=1)
    subj, acts, ml = W.intents_workload(n, s, rounds, rate=0.05, seed=79)
    g, w = pair(cfg, subj, W.initial_views(s))
    g.set_checker(period, mx, 0, 128)
    L.orc_world_set_checker(C.byref(w), mx, 0, 128, period)
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t], threads=16)
        if (t + 1) % 5 == 0:
            same(g, w, f"round {t}")
    got = g.checker_stats()
    assert list(got["queued"]) + list(got["warn"]) + list(got["pruned"]) == list(w.chk_stats)
    assert int(w.chk_stats[6]) > 0
    st = H.engine_state(g, H.world_width(w))
    assert int(st["q_pruned"].sum()) == 0 and int(st["q_expired"].sum()) == 0
    g.close()
    L.orc_world_free(C.byref(w))


@pytest.mark.parametrize("qcap,depth,mn", [(16, 100, 0), (32, 0, 0), (16, 100, 5)])
def test_in_round_checker_churn_bit_exact(qcap, depth, mn):
    """In-round ticks over all three queues with churn (members going down keep their pending
    re-queues: the tick's flush applies them before the fork), deep and bounded queues, and
    the per-member max (min_queue_depth > 0: queue_max_kernel reads the views before the
    merge changes them); bit-exact every round."""
    n, rounds, period = 1200, 20, 4
    subj, acts, ml = W.churn_workload(n, rounds, events_per_round=30, queries_per_round=5, seed=qcap + depth + mn)
    s = len(subj)
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=qcap, queue_depth=(depth, depth, depth),
                         gossip_limit=400, gossip_overhead=3, retransmit_mult=4, max_rumors=512,
                         event_buffer_size=128, query_buffer_size=128, slot_k=8, max_refute=2)
    g, w = pair(cfg, subj, W.initial_views(s))
    mx = max(4, (depth or qcap) // 3)
    g.set_checker(period, mx, mn, 8)
    L.orc_world_set_checker(C.byref(w), mx, mn, 8, period)
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t])
        same(g, w, f"round {t}")
    got = g.checker_stats()
    assert list(got["queued"]) + list(got["warn"]) + list(got["pruned"]) == list(w.chk_stats)
    if not mn:
        assert int(sum(w.chk_stats[6:9])) > 0
    g.set_checker(0)
    g.close()
    L.orc_world_free(C.byref(w))


@pytest.mark.parametrize("qcap,depth", [(16, 100), (32, 0)])
def test_staggered_ticks_churn_bit_exact(qcap, depth):
    """Phased ticks over all three queues with churn, deep (head + tail) and bounded queues:
    each round's phase of 4 prunes to a max small enough to bite; bit-exact every round."""
    n, rounds, period = 1200, 20, 4
    subj, acts, ml = W.churn_workload(n, rounds, events_per_round=30, queries_per_round=5, seed=qcap + depth)
    s = len(subj)
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=qcap, queue_depth=(depth, depth, depth),
                         gossip_limit=400, gossip_overhead=3, retransmit_mult=4, max_rumors=512,
                         event_buffer_size=128, query_buffer_size=128, slot_k=8, max_refute=2)
    g, w = pair(cfg, subj, W.initial_views(s))
    mx = max(4, (depth or qcap) // 3)
    pruned = 0
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t])
        g.check_queues_phase(period, t % period, mx, 0, 8)
        exp = (C.c_uint64 * 9)()
        L.orc_check_queues_phase(C.byref(w), mx, 0, 8, period, t % period, exp)
        pruned += sum(exp[6:9])
        same(g, w, f"round {t}")
    assert pruned > 0
    with pytest.raises(Exception):
        g.check_queues_phase(4, 4)
    g.close()
    L.orc_world_free(C.byref(w))


@pytest.mark.parametrize("qcap,depth,limit,mult", [(16, 100, 400, 4), (64, 200, 260, 1), (8, 40, 600, 2),
                                                   (32, 64, 1400, 4)])
def test_deep_churn_flood_prune_ring_bit_exact(qcap, depth, limit, mult):
    """Intents, user events and queries of many lengths with churn, through heads of 8..64
    slots and depths small enough to fill: spills, the deferred whole-queue emissions, the
    bounded prune at the full depth (the largest key of head and tail, which the spills put
    in the tail: deep_prune_wave / tail_prune_serial), retransmit
    limits of 1..4 (items retiring out of the head), a rumor ring small enough to wrap (tail
    items expire), and QueueChecker ticks.  Bit-exact against the oracle after every round."""
    n, rounds = 1200, 30
    subj, acts, ml = W.churn_workload(n, rounds, events_per_round=30, queries_per_round=5, seed=depth + qcap)
    s = len(subj)
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=qcap, queue_depth=(depth, depth, depth),
                         gossip_limit=limit, gossip_overhead=3, retransmit_mult=mult, max_rumors=512,
                         event_buffer_size=128, query_buffer_size=128, slot_k=8, max_refute=2)
    g, w = pair(cfg, subj, W.initial_views(s))
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t])
        same(g, w, f"round {t}")
        if t in (9, 19):
            check_both(g, w, depth // 2, 0, 8, f"round {t}")
    total, _ = g.deep_stats()
    assert total > 0
    assert w.gen >= 2
    check_both(g, w, 4096, 0, 128, "end")
    check_both(g, w, 5, 0, 2, "end")
    g.close()
    L.orc_world_free(C.byref(w))


def test_deep_serial_inserts_and_prune():
    """A member whose peers are all down sends nothing, so its own originations pile up in its
    pending list; at 128 entries the list is applied one item at a time (pend_push_serial ->
    queue_insert_item): the full head's largest falls into the tail, and past the depth the
    largest key of head and tail is pruned (tail_prune_serial).  200 user events of many
    lengths through a head of 8 and a depth of 40; compared with the oracle's queue at the end
    (an inspection applies the list, so it would hide the serial path if done every round)."""
    n, rounds = 3, 200
    cfg = G.GossipConfig(n_members=n, n_subjects=1, queue_cap=8, queue_depth=(40, 40, 40), fanout=1,
                         max_rumors=1 << 12, event_buffer_size=512, query_buffer_size=64, slot_k=4)
    subj = np.array([2], np.uint32)
    g, w = pair(cfg, subj, W.initial_views(1))
    alive = np.array([1, 0, 0], np.uint8)
    g.set_alive(alive)
    for m in range(n):
        w.alive[m] = int(alive[m])
    rng = np.random.default_rng(3)
    for t in range(rounds):
        acts = np.zeros(1, G.ACTION_DTYPE)
        acts["member"], acts["act"] = 0, G.ACT_USER_EVENT
        acts["name_len"], acts["payload_len"] = rng.integers(1, 30), rng.integers(0, 60)
        acts["key"] = (int(rng.integers(1, 9)) << 32) | int(rng.integers(1, 99))
        g.round(t, None, acts)
        H.oracle_round(w, t, np.zeros(0, G.ML_DTYPE), acts)
    same(g, w, "end")
    assert int(g.pruned()[0]) == rounds - 40 and O.arr(w.q_pruned, n, np.uint32)[0] == rounds - 40
    g.close()
    L.orc_world_free(C.byref(w))


def test_configs3_100k_deep_queues_bit_exact():
    """BASELINE configs[3] (100k members, 1% churn, 100 user events + 10 queries per round)
    with all three queues 4096 deep: every member's clocks, digest of every delivery, error
    bits and queue drops bit-exact every round, the full state (queues included) at the end."""
    n, rounds = 100_000, 9
    subj, acts, ml = W.churn_workload(n, rounds, events_per_round=100, queries_per_round=10, seed=2024)
    s = len(subj)
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=64, queue_depth=(4096, 4096, 4096), gossip_limit=1400,
                         max_rumors=1 << 16, event_buffer_size=512, query_buffer_size=512, slot_k=16)
    g, w = pair(cfg, subj, W.initial_views(s))
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t], threads=16)
        m = g.members()
        for k, ok in [("clock", w.clock), ("event_clock", w.eclock), ("query_clock", w.qclock),
                      ("digest", w.digest), ("err", w.err)]:
            exp = O.arr(ok, n, np.uint32 if k == "err" else np.uint64)
            assert np.array_equal(m[k], exp), (t, k)
        assert np.array_equal(g.pruned(), O.arr(w.q_pruned, n, np.uint32)), t
    same(g, w, "final")
    assert int(g.pruned().sum()) == 0
    total, _ = g.deep_stats()
    assert total > 0
    g.close()
    L.orc_world_free(C.byref(w))


@pytest.mark.parametrize("checker", [False, True])
def test_deep_two_shards_buckets_equal_one_context(checker):
    """The multi-GPU bucket emission with deep queues (emit_kernel_deep and the deferred classes
    writing into the destination buckets): two shard contexts on one GPU, the exchange by hand,
    equal to one context after every round; with `checker`, the in-round staggered ticks too
    (phases by global member id, so each shard ticks its own members of that phase)."""
    import torch
    from ruserf_amd.dist import hbm_tensor
    n, rounds = 4000, 12
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    subj, acts, ml = W.churn_workload(n, rounds, events_per_round=40, queries_per_round=6, seed=9)
    s = len(subj)
    base = dict(n_members=n, n_subjects=s, queue_cap=16, queue_depth=(300, 300, 300), gossip_limit=500,
                max_rumors=1 << 16, event_buffer_size=128, query_buffer_size=128, slot_k=8)
    views = W.initial_views(s)
    one = G.GossipEngine(G.GossipConfig(**base))
    shards = [G.GossipEngine(G.GossipConfig(**base, shard=(0, n // 2))),
              G.GossipEngine(G.GossipConfig(**base, shard=(n // 2, n)))]
    for e in [one] + shards:
        e.set_stream(stream.cuda_stream)
        e.set_subjects(subj)
        e.init_views(*views)
        if checker:
            e.set_checker(3, 40, 0, 8)
    bufs = [e.bucket_buffers(2) for e in shards]
    words = bufs[0][2] // 4
    for t in range(rounds):
        one.round(t, ml[t], acts[t])
        for e in shards:
            e.round_begin(t, ml[t], acts[t])
        blocks = [hbm_tensor(*e.rumor_block()[:1], e.rumor_block()[1] // 8) for e in shards]
        total = blocks[0] + blocks[1]
        for b in blocks:
            b.copy_(total)
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
        width = 300
        full = H.normalize_queues(H.engine_state(one, width))
        halves = [H.normalize_queues(H.engine_state(e, width)) for e in shards]
        for k in full:
            assert np.array_equal(np.concatenate([halves[0][k], halves[1][k]]), full[k]), (t, k)
    assert sum(e.deep_stats()[0] for e in shards) > 0
    if checker:
        got = [e.checker_stats() for e in [one] + shards]
        for key in ("queued", "warn", "pruned"):
            assert np.array_equal(got[0][key], got[1][key] + got[2][key]), key
        assert int(got[0]["pruned"].sum()) > 0
    for e in [one] + shards:
        e.close()


@pytest.mark.parametrize("depth,rounds", [(2500, 34), (1400, 40), (2600, 90)])
def test_deep_long_queues_all_capacity_classes(depth, rounds):
    """Queues that grow past the deferred path's two smaller LDS capacities (832 and 1 216
    items): a user-event flood (100 per round) that the retransmit limit retires far slower
    than it arrives, an event buffer wide enough to accept every event, and a rumor ring that
    does not wrap, so the event queues of every member grow by tens of items per round.  Members
    deferred at every size class take emit_deep_wave_kernel<832>, <1216> and the block classes
    (emit_deep_block_kernel<2432> and the full depth); bit-exact against the oracle every third
    round, with the largest queue past 1 216 items by the end.  Depth 2 500: nothing pruned;
    1 400 and 2 600: the event queues reach their depth inside the middle class and the full
    depth, so the block classes' bounded prune runs (drops counted, equal to the oracle's)."""
    n = 300
    subj, acts, ml = W.churn_workload(n, rounds, churn=0.01, events_per_round=100, queries_per_round=0, seed=77)
    s = len(subj)
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=64, queue_depth=(depth, depth, depth), gossip_limit=1000,
                         gossip_overhead=2, retransmit_mult=4, max_rumors=1 << 17, event_buffer_size=10000,
                         query_buffer_size=64, slot_k=16, max_refute=2)
    g, w = pair(cfg, subj, W.initial_views(s))
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t], threads=16)
        if t % 3 == 2 or t == rounds - 1:
            same(g, w, f"round {t}")
    assert H.world_width(w) > 1216  # queues past the two smaller capacity classes
    total, _ = g.deep_stats()
    assert total > 0
    cls = g.deep_class_stats()
    assert cls[2] > 0, cls  # the middle class ran
    if depth == 2500:
        assert int(g.pruned().sum()) == 0
    else:
        assert int(g.pruned().sum()) > 0  # the bounded prune at the depth ran
    if depth == 2600:
        assert cls[3] > 0, cls  # the full depth ran
    g.close()
    L.orc_world_free(C.byref(w))


@pytest.mark.parametrize("qcap,depth", [(16, 100), (64, 130)])
def test_deep_intent_only_prune_bit_exact(qcap, depth):
    """Only the intent queue deep (queue_depth = (d, 0, 0)) and small enough to overflow:
    the intent-only emission (emit_kernel_deep<..., 1u>, the other queues' tail code compiled
    away) and the bounded prune at the depth inside emit_deep_wave_kernel.  The saturated
    intent workload, bit-exact against the oracle after every round, drops counted."""
    n, s, rounds = 4000, 1024, 14
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=qcap, queue_depth=(depth, 0, 0), gossip_limit=8 * 24,
                         gossip_overhead=2, max_rumors=1 << 16, event_buffer_size=512, query_buffer_size=512,
                         slot_k=1)
    subj, acts, ml = W.intents_workload(n, s, rounds, rate=0.05, seed=5)
    g, w = pair(cfg, subj, W.initial_views(s))
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t], threads=16)
        same(g, w, f"round {t}")
    assert int(g.pruned().sum()) > 0  # the depth was reached
    total, _ = g.deep_stats()
    assert total > 0
    g.close()
    L.orc_world_free(C.byref(w))


def test_configs1_reference_regime_properties():
    """BASELINE configs[1] (1M members, 4096 tracked subjects) in the bench's reference regime:
    the intent queue 8704 deep, in-round staggered ticks to 4096 every 150 rounds, the ring
    sized so nothing expires, 320 rounds (every member ticked at least once past 4096 items).
    Too large for the oracle, so size-independent properties: nothing dropped between ticks
    and nothing expired; no capacity error; each tick of the last round pruned to exactly the
    max (pruned = queued - 4096 x members ticked, from the checker's own counts, none below
    it); those members hold at most the max plus the round's re-queues, every queue at most
    its depth; the items queued stay under the retransmit limit; the hipCUB temporaries
    intact."""
    n, s, rounds, period, mx = 1_000_000, 4096, 320, 150, 4096
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=64, queue_depth=(8704, 0, 0), gossip_limit=8 * 24,
                         gossip_overhead=2, max_rumors=1 << 23, event_buffer_size=512, query_buffer_size=512,
                         slot_k=1)
    subj, acts, ml = W.intents_workload(n, s, rounds, rate=0.01, seed=0x5EED, prune_frac=0.1)
    g = G.GossipEngine(cfg)
    g.set_subjects(subj)
    g.init_views(*W.initial_views(s))
    g.set_checker(period, mx, 0, 128)
    for t in range(rounds - 1):
        g.round(t, ml[t], acts[t])
    g.checker_stats(reset=True)
    t = rounds - 1
    g.round(t, ml[t], acts[t])
    st = g.checker_stats()
    occ = g.checker_occupancy()
    ticked = int(occ["hist"][0].sum())
    assert ticked == len(range(t % period, n, period))
    over = int(st["warn"][0])  # every ticked member is over the warning depth (128)
    assert over == ticked and int(st["pruned"][0]) > 0
    # no ticked queue below the max: each was pruned to exactly the max
    assert int(occ["hist"][0][:mx // occ["bin"]].sum()) == 0
    assert int(st["pruned"][0]) == int(st["queued"][0]) - mx * ticked
    # (read after the round's merge, whose re-queues the read applies first: at most one
    # pending list of 128 entries on top of the pruned 4096)
    ql = g.queue_lengths()[:, 0].astype(np.int64)
    assert np.all(ql[t % period::period] <= mx + 128)
    assert np.median(ql) > mx + 128  # the others are not
    assert int(ql.max()) <= cfg.depths()[0]
    assert int(g.pruned().sum()) == 0 and int(g.expired().sum()) == 0
    m = g.members()
    assert np.all((m["err"] & ~np.uint32(G.E_QUEUE_PRUNE)) == 0) and np.all(m["err"] == 0)
    rows = (0, 64)
    r, sq, tx, ln = g.queues_rows(rows[0], rows[1], cfg.depths()[0])
    limit = O.lib().orc_retransmit_limit(4, n)
    assert np.all(tx[r != 0xFFFFFFFF] < limit)
    assert all(g.cub_canaries())
    g.close()


def test_packed_intent_tail_config_limits():
    """The intent queue's packed 8-B tail items hold the rumor's ring slot and
    generation parity in 27 bits and transmits in 6: a deep intent queue with more than 2^26
    ring slots per generation or a retransmit limit above 64 is refused at create, and the
    same configurations with a bounded (or query/event-only deep) queue are accepted."""
    base = dict(n_members=64, n_subjects=4, queue_cap=16, event_buffer_size=16, query_buffer_size=16, slot_k=2)
    with pytest.raises(Exception):
        G.GossipEngine(G.GossipConfig(**base, queue_depth=(100, 0, 0), max_rumors=1 << 27))
    with pytest.raises(Exception):
        G.GossipEngine(G.GossipConfig(**base, queue_depth=(100, 0, 0), retransmit_mult=33, max_rumors=1 << 10))
    for cfg in [G.GossipConfig(**base, max_rumors=1 << 27),
                G.GossipConfig(**base, queue_depth=(0, 100, 100), retransmit_mult=33, max_rumors=1 << 10),
                G.GossipConfig(**base, queue_depth=(100, 0, 0), max_rumors=1 << 26)]:
        G.GossipEngine(cfg).close()


def test_view_time_stamps_mod_2_27_reaper_ages():
    """View time stamps are kept mod 2^27 rounds (12-B view entries): a Left
    member stamped just below 2^27 and reaped just above it ages by the true difference, so the
    Reaper's tombstone decision equals the oracle's (which keeps the whole u32)."""
    n, s = 8, 2
    subj = np.array([6, 7], np.uint32)
    for timeout, reaped in [(25, True), (35, False)]:
        cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=8, max_rumors=1024, event_buffer_size=64,
                             query_buffer_size=64, slot_k=2)
        g, w = pair(cfg, subj, W.initial_views(s))
        stamp, now = (1 << 27) - 10, (1 << 27) + 20  # true age 30 rounds
        for m in range(n):  # every member knows subject 0 as Leaving
            g.set_view(m, 0, G.KIND_KNOWN, G.STATUS_LEAVING, 3)
        O.arr(w.v_kind, n * s, np.uint8).reshape(n, s)[:, 0] = G.KIND_KNOWN
        O.arr(w.v_status, n * s, np.uint8).reshape(n, s)[:, 0] = G.STATUS_LEAVING
        O.arr(w.v_ltime, n * s, np.uint64).reshape(n, s)[:, 0] = 3
        # memberlist NotifyLeave of subject 0 at round `stamp`: Leaving -> Left, leave_time = stamp
        ml = np.zeros(1, G.ML_DTYPE)
        ml["subject"], ml["kind"], ml["set_alive"] = 0, G.ML_LEAVE, 2  # (liveness unchanged)
        g.round(stamp, ml, None)
        H.oracle_round(w, stamp, ml, np.zeros(0, G.ACTION_DTYPE))
        _, st, kd, tm = g.view(with_time=True)
        assert int(st.reshape(n, s)[1, 0]) == G.STATUS_LEFT and int(tm.reshape(n, s)[1, 0]) == stamp % (1 << 27)
        g.reap(now, 1 << 30, timeout, 1 << 30)
        assert L.orc_reap(C.byref(w), now, 1 << 30, timeout, 1 << 30) == 0
        _, st, kd, tm = g.view(with_time=True)
        exp_kind = O.arr(w.v_kind, n * s, np.uint8).reshape(n, s)
        assert np.array_equal(kd.reshape(n, s), exp_kind)
        assert (int(exp_kind[1, 0]) == G.KIND_UNKNOWN) == reaped, (timeout, exp_kind[1, 0])
        g.close()
        L.orc_world_free(C.byref(w))
