"""The bench's own queue regime, bit-exact against the oracle at the bench's own parameters.

bench.py's gossip line runs the reference's queue regime: the intent queue
8 704 deep, each member's QueueChecker ticking on its own phase every 150 rounds (in round r the
members with id = r mod 150, between the emission and the merge) and pruning its queue to
max_queue_depth 4096 (core/src/serf/base.rs:703-760, core/src/options.rs:249, 512), the ring
sized so nothing expires, settled 330 rounds so the queues sit at their steady state (4-8.4k
items).  The 1M-member line is too large for the oracle, so this test runs the same regime --
the same workload shape (4096 tracked subjects, 1% of members originating per round, 8 intents
of budget per target, fanout 3), the same depth, checker period, max and warning -- at 12k
members for 340 rounds, where the queues reach the bench's occupancy (experiments/
regime_small.py: mean 5.8k, p99 7.6k, max 7.8k items at the end), and compares the engine with
the oracle: every member's clocks, digest, errors, views, dedup rings and queue bookkeeping
every 10 rounds, the queues of a rotating block of members every 10 rounds, the checker's
counts, and every queue of every member after the last round.

It asserts that each path the 1M line runs ran here too: all four LDS classes of the deferred
whole-queue emission, the full-depth class on queues of more than 4096 items,
check_stream_kernel's select over more than 4096 keys, and sealed tail prefixes of more than
4000 items."""
import ctypes as C

import numpy as np
import pytest

import gossip_harness as H
import oracle_ffi as O
from ruserf_amd import gossip as G
from ruserf_amd import workload as W

pytestmark = pytest.mark.gpu
L = O.lib()

N, S, ROUNDS, PERIOD, MX, WARN, DEPTH, RATE = 12_000, 4096, 340, 150, 4096, 128, 8704, 0.01
BLOCK = 1000  # members whose queues are compared every 10 rounds (rotating)


def ring_for(n, rounds):
    per_round = S * 4 + int(round(n * RATE))
    return 1 << max(10, (per_round * rounds - 1).bit_length())


def intent_queue_canonical(r, sq, tx, ln):
    """one queue's items per row sorted by the send-order key, empty slots last and zeroed"""
    r, sq, tx, ln = (np.asarray(a) for a in (r, sq, tx, ln))
    empty = r == 0xFFFFFFFF
    key = (tx.astype(np.uint64) << np.uint64(48)) | ((np.uint64(0xFFFF) - ln.astype(np.uint64)) << np.uint64(32)) \
        | (np.uint64(0xFFFFFFFF) - sq.astype(np.uint64))
    key = np.where(empty, np.uint64(0xFFFFFFFFFFFFFFFF), key)
    order = np.argsort(key, axis=1, kind="stable")
    out = []
    for a in (r, sq, tx, ln):
        b = np.take_along_axis(a, order, axis=1).copy()
        if a is not r:
            b[np.take_along_axis(empty, order, axis=1)] = 0
        out.append(b)
    return out


def compare_queues(g, w, lo, hi, width, ctx):
    r, sq, tx, ln = g.queues_rows(lo, hi - lo, width)
    o = H.world_state(w, lo, hi, width=width)
    o_r, o_sq, o_tx, o_ln = (o[k].reshape(hi - lo, 3, width) for k in ("q_rumor", "q_seq", "q_tx", "q_len"))
    for q in range(3):
        got = intent_queue_canonical(r[:, q], sq[:, q], tx[:, q], ln[:, q])
        exp = intent_queue_canonical(o_r[:, q], o_sq[:, q], o_tx[:, q], o_ln[:, q])
        for name, a, b in zip(("rumor", "seq", "tx", "len"), got, exp):
            if not np.array_equal(a, b):
                bad = np.argwhere(a != b)
                raise AssertionError(f"{ctx}: queue {q} {name} differs at {len(bad)} places, first row "
                                     f"{lo + int(bad[0][0])}: got {a[tuple(bad[0])]} expected {b[tuple(bad[0])]}")


def compare_members(g, w, ctx):
    m = g.members()
    for k, p, t in [("clock", w.clock, np.uint64), ("event_clock", w.eclock, np.uint64),
                    ("query_clock", w.qclock, np.uint64), ("digest", w.digest, np.uint64),
                    ("err", w.err, np.uint32), ("serf_state", w.serf_state, np.uint8)]:
        assert np.array_equal(m[k], O.arr(p, N, t)), (ctx, k)
    assert np.array_equal(g.pruned(), O.arr(w.q_pruned, N, np.uint32)), ctx
    assert np.array_equal(g.expired(), O.arr(w.q_expired, N, np.uint32)), ctx
    lt, st, kd, vt = g.view(with_time=True)
    for name, a, p, t in [("ltime", lt, w.v_ltime, np.uint64), ("status", st, w.v_status, np.uint8),
                          ("kind", kd, w.v_kind, np.uint8), ("time", vt, w.v_time, np.uint32)]:
        assert np.array_equal(a.reshape(N, S), O.arr(p, N * S, t).reshape(N, S)), (ctx, "view", name)
    ebl, ebc, ebk, qbl, qbc, qbi = g.buffers()
    for name, a, p, t in [("eb_ltime", ebl, w.eb_ltime, np.uint64), ("eb_cnt", ebc, w.eb_cnt, np.uint32),
                          ("eb_keys", ebk, w.eb_keys, np.uint64), ("qb_ltime", qbl, w.qb_ltime, np.uint64),
                          ("qb_cnt", qbc, w.qb_cnt, np.uint32), ("qb_ids", qbi, w.qb_ids, np.uint32)]:
        a = np.asarray(a).reshape(-1)
        assert np.array_equal(a, O.arr(p, a.size, t)), (ctx, name)


@pytest.mark.timeout(1500)
def test_bench_regime_bit_exact():
    cfg = G.GossipConfig(n_members=N, n_subjects=S, queue_cap=64, queue_depth=(DEPTH, 0, 0), gossip_limit=8 * 24,
                         gossip_overhead=2, retransmit_mult=4, max_rumors=ring_for(N, ROUNDS),
                         event_buffer_size=512, query_buffer_size=512, slot_k=1, fanout=3, max_refute=4)
    subj, acts, ml = W.intents_workload(N, S, ROUNDS, rate=RATE, seed=0x5EED, prune_frac=0.1)
    views = W.initial_views(S)
    g = G.GossipEngine(cfg)
    g.set_subjects(subj)
    g.init_views(*views)
    w = H.oracle_world(cfg, subj, views)
    g.set_checker(PERIOD, MX, 0, WARN)
    L.orc_world_set_checker(C.byref(w), MX, 0, WARN, PERIOD)
    cls0 = g.deep_class_stats()
    sealed_max, blk = 0, 0
    for t in range(ROUNDS):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t], threads=16)
        _, sealed = g.tails(0)  # (no flush: the tails as the emission left them)
        sealed_max = max(sealed_max, int(sealed.max()))
        if (t + 1) % 10 == 0:
            compare_members(g, w, f"round {t}")
            lo = (blk * BLOCK) % N
            compare_queues(g, w, lo, min(N, lo + BLOCK), H.world_width(w), f"round {t}")
            blk += 1
            print(f"regime round {t}: equal (queue width {H.world_width(w)})", flush=True)  # progress
    ctx = "after the last round"
    compare_members(g, w, ctx)
    width = H.world_width(w)
    for lo in range(0, N, 2000):
        compare_queues(g, w, lo, min(N, lo + 2000), width, ctx)
    got = g.checker_stats()
    assert list(got["queued"]) + list(got["warn"]) + list(got["pruned"]) == list(w.chk_stats)
    # the regime: nothing dropped between ticks, nothing expired, no capacity error; the ticks pruned
    assert int(g.pruned().sum()) == 0 and int(g.expired().sum()) == 0
    assert np.all(g.members()["err"] == 0)
    assert int(w.chk_stats[6]) > 0
    # the queues at the bench's occupancy
    ql = g.queue_lengths()[:, 0].astype(np.int64)
    assert ql.mean() > 5000 and int(ql.max()) > 7000, (ql.mean(), ql.max())
    # every path of the 1M line ran: the four deferred classes ...
    cls = g.deep_class_stats() - cls0
    assert np.all(cls > 0), cls
    # ... the full-depth class on queues of more than 4096 items ...
    fsum, fmax = g.deep_full_items()
    assert fmax > 4096, (fsum, fmax)
    # ... the checker's select over more than 4096 keys (a tick's occupancy before its prune) ...
    assert int(g.checker_occupancy()["max"][0]) > 4096
    # ... and sealed tail prefixes past 4k items
    assert sealed_max > 4000, sealed_max
    g.close()
    L.orc_world_free(C.byref(w))
