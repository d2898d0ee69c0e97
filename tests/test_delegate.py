"""MergeDelegate::notify_merge (core/src/delegate/merge.rs:13-28) as the engine's host
hook: a cancelled alive merge yields no NotifyJoin, a cancelled join push/pull no merge
(CPU: the host filter plus the oracle world it feeds)."""
import ctypes as C

import numpy as np

import gossip_harness as H
import oracle_ffi as O
from ruserf_amd import gossip as G
from ruserf_amd import workload as W
from ruserf_amd.delegate import (DefaultMergeDelegate, Member, MergeCanceled, MergeDelegate,
                                 filter_alive_events, filter_join_push_pull)

L = O.lib()


class RejectSubjects(MergeDelegate):
    def __init__(self, banned):
        self.banned, self.calls = set(banned), 0

    def notify_merge(self, members):
        self.calls += 1
        if any(m.subject in self.banned for m in members):
            raise MergeCanceled("banned node")


def _ml(rows):
    out = np.zeros(len(rows), dtype=G.ML_DTYPE)
    for i, (s, k, a) in enumerate(rows):
        out[i] = (s, k, a, 0)
    return out


def test_filter_alive_events_drops_cancelled_joins_only():
    subj = np.array([10, 20, 30, 40], np.uint32)
    ml = _ml([(0, G.ML_JOIN, 1), (1, G.ML_LEAVE, 0), (2, G.ML_JOIN, 1), (3, G.ML_UPDATE, 2), (2, G.ML_LEAVE, 2)])
    d = RejectSubjects({2})
    out = filter_alive_events(d, ml, subj)
    assert d.calls == 2  # one notify_merge per alive (JOIN) event
    assert out["subject"].tolist() == [0, 1, 3, 2] and out["kind"].tolist() == [G.ML_JOIN, G.ML_LEAVE,
                                                                                  G.ML_UPDATE, G.ML_LEAVE]
    assert len(filter_alive_events(DefaultMergeDelegate(), ml, subj)) == len(ml)


def test_filter_join_push_pull_consults_remote_nodes():
    pairs = np.zeros(3, dtype=G.PP_PAIR_DTYPE)
    pairs["receiver"] = [1, 2, 3]
    pairs["sender"] = [7, 8, 9]
    remote = {7: [Member(0, 100)], 8: [Member(0, 100), Member(5, 105)], 9: []}
    out = filter_join_push_pull(RejectSubjects({5}), pairs, lambda s: remote[s])
    assert out["sender"].tolist() == [7, 9]


def test_cancelled_rejoin_keeps_member_failed_in_views():
    n, s = 400, 8
    subj = np.arange(0, 2 * s, 2, dtype=np.uint32)
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=16, gossip_limit=400, max_rumors=1 << 12,
                         event_buffer_size=32, query_buffer_size=32, slot_k=4)
    w = H.oracle_world(cfg, subj, W.initial_views(s))
    none = np.zeros(0, dtype=G.ACTION_DTYPE)
    H.oracle_round(w, 0, _ml([(3, G.ML_LEAVE, 2), (4, G.ML_LEAVE, 2)]), none)
    ml = filter_alive_events(RejectSubjects({4}), _ml([(3, G.ML_JOIN, 2), (4, G.ML_JOIN, 2)]), subj)
    H.oracle_round(w, 1, ml, none)
    st = O.arr(w.v_status, n * s, np.uint8).reshape(n, s)
    others = np.setdiff1d(np.arange(n), subj[[3, 4]])
    assert np.all(st[others, 3] == O.ST_ALIVE) and np.all(st[others, 4] == O.ST_FAILED)
    L.orc_world_free(C.byref(w))
