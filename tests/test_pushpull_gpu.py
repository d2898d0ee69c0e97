"""Push/pull anti-entropy (SerfDelegate::local_state / merge_remote_state,
core/src/serf/delegate.rs:376-554) on the GPU against the oracle, bit for bit:
clocks, views, event dedup rings, member-event / delivery digests, refutations.
The oracle's merge is pinned by the reference's delegate_merge_remote_state KAT
(tests/test_oracle_kat.py)."""
import ctypes as C

import numpy as np
import pytest

import gossip_harness as H
import oracle_ffi as O
from ruserf_amd import gossip as G
from ruserf_amd import workload as W

L = O.lib()


def _world(n, rounds, seed):
    cfg = G.GossipConfig(n_members=n, n_subjects=max(2, n // 100), queue_cap=32, gossip_limit=400,
                         max_rumors=1 << 16, event_buffer_size=128, query_buffer_size=128, slot_k=4)
    subj, acts, ml = W.churn_workload(n, rounds + 4, events_per_round=25, queries_per_round=3, seed=seed)
    views = W.initial_views(len(subj))
    return cfg, subj, acts, ml, views


@pytest.mark.gpu
@pytest.mark.parametrize("n,rounds,flags", [(1200, 8, (False, False)), (2000, 10, (True, True)),
                                            (900, 6, (True, False))])
def test_push_pull_bit_exact(n, rounds, flags):
    cfg, subj, acts, ml, views = _world(n, rounds, seed=31 + n)
    g = G.GossipEngine(cfg)
    g.set_subjects(subj)
    g.init_views(*views)
    w = H.oracle_world(cfg, subj, views)
    rng = np.random.default_rng(n)
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t])
        if t % 2 == 1:
            # a symmetric exchange between half of the members, plus one-sided pulls
            members = rng.choice(n, size=n // 2, replace=False)
            pairs = H.matching_pairs(rng, members)
            rest = np.setdiff1d(np.arange(n), pairs["receiver"])[: n // 8]
            one = np.zeros(len(rest), G.PP_PAIR_DTYPE)
            one["receiver"] = rest
            one["sender"] = rng.integers(0, n, size=len(rest))
            pairs = np.concatenate([pairs, one])
            g.push_pull(pairs, *flags)
            H.oracle_push_pull(w, pairs, *flags)
        H.assert_same(H.engine_state(g), H.world_state(w), f"round {t}")
    st = H.engine_state(g)
    assert np.any(st["eb_cnt"] > 0)
    g.close()
    L.orc_world_free(C.byref(w))


@pytest.mark.gpu
def test_push_pull_rejects_repeated_receiver():
    cfg, subj, _, _, views = _world(300, 2, seed=5)
    g = G.GossipEngine(cfg)
    g.set_subjects(subj)
    g.init_views(*views)
    pairs = np.zeros(2, G.PP_PAIR_DTYPE)
    pairs["receiver"] = [3, 3]
    pairs["sender"] = [4, 5]
    with pytest.raises(RuntimeError):
        g.push_pull(pairs)
    g.close()


def test_oracle_push_pull_snapshot_semantics():
    """A symmetric exchange merges each side's PRE-exchange state (memberlist sends its
    local state before merging the remote one): after a<->b both hold the max clock."""
    cfg, subj, _, _, views = _world(200, 2, seed=9)
    w = H.oracle_world(cfg, subj, views)
    w.clock[10], w.clock[20] = 50, 7
    w.eclock[10], w.eclock[20] = 3, 90
    pairs = np.zeros(2, G.PP_PAIR_DTYPE)
    pairs["receiver"] = [10, 20]
    pairs["sender"] = [20, 10]
    H.oracle_push_pull(w, pairs)
    # witness(t - 1): c = max(c, t)
    assert (w.clock[10], w.clock[20]) == (50, 50)
    assert (w.eclock[10], w.eclock[20]) == (90, 90)
    L.orc_world_free(C.byref(w))
