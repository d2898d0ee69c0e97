"""The snapshot log and the Reconnector on the CPU oracle (test infrastructure).

The first tests restate the reference's own snapshotter unit tests
(core/src/serf/base/tests/serf/snapshot.rs: snapshoter, snapshoter_force_compact,
snapshoter_leave, snapshoter_leave_rejoin) against the oracle's in-memory
Snapshotter; a node "foo" is subject 7 (the model's node identity is the subject).
The world tests check the per-member snapshotters that the engine mirrors: the
encoded file replays to the member's live alive set and clocks, a restart from it
witnesses the clocks and refuses re-delivery of older events (serf_snapshot_recovery,
same file), and the Reconnector only ever targets failed members.
"""
import ctypes as C

import numpy as np
import pytest

import gossip_harness as H
import oracle_ffi as O
from ruserf_amd import gossip as G
from ruserf_amd import workload as W

L = O.lib()
S = 64
FOO = 7
EV_JOIN, EV_LEAVE, EV_FAILED = 0, 1, 2
SNAPSHOT_SIZE_LIMIT = 128 * 1024  # snapshot.rs test constant (min_compact_size)


def u8(b):
    a = np.frombuffer(bytes(b), dtype=np.uint8).copy() if len(b) else np.zeros(1, np.uint8)
    return a


def replay(data, rejoin=False, s=S):
    a = u8(data)
    bits = np.zeros((s + 31) // 32, np.uint32)
    clocks = np.zeros(3, np.uint64)
    rc = L.orc_snapshot_replay(O.ptr(a, C.c_uint8), len(data), int(rejoin), s, O.ptr(bits, C.c_uint32),
                               O.ptr(clocks, C.c_uint64))
    alive = {i for i in range(s) if bits[i >> 5] >> (i & 31) & 1}
    return rc, alive, [int(x) for x in clocks]


class Snap:
    def __init__(self, data=b"", min_compact=SNAPSHOT_SIZE_LIMIT, rejoin=False):
        self.sp = O.Snapshotter()
        a = u8(data)
        assert L.orc_snapshotter_open(C.byref(self.sp), S, O.ptr(a, C.c_uint8), len(data), min_compact,
                                      int(rejoin)) == 0
        self.clock = 0  # a LamportClock::new() shared with the snapshotter

    def witness(self, t):
        if t >= self.clock:
            self.clock = t + 1

    def user(self, lt):
        L.orc_snapshotter_user_event(C.byref(self.sp), lt)

    def query(self, lt):
        L.orc_snapshotter_query(C.byref(self.sp), lt)

    def member(self, ev, subj):
        L.orc_snapshotter_member_event(C.byref(self.sp), ev, subj, self.clock)

    def leave(self):
        L.orc_snapshotter_leave(C.byref(self.sp))

    def close(self):
        """shutdown: the stream's final update_clock, then the file"""
        L.orc_snapshotter_update_clock(C.byref(self.sp), self.clock)
        data = bytes(np.ctypeslib.as_array(self.sp.buf, (self.sp.len,))) if self.sp.len else b""
        L.orc_snapshotter_free(C.byref(self.sp))
        return data


def test_snapshoter_kat():
    """snapshot.rs tests: snapshoter -- ue 42, query 50, clock witness 100, foo join /
    failed / join; replay gives clocks (100, 42, 50) and foo alive."""
    s = Snap()
    s.user(42)
    s.query(50)
    s.witness(100)
    s.member(EV_JOIN, FOO)
    s.member(EV_FAILED, FOO)
    s.member(EV_JOIN, FOO)
    data = s.close()
    rc, alive, clocks = replay(data)
    assert rc == 0 and clocks == [100, 42, 50] and alive == {FOO}
    # reopen and close again: nothing new is appended and the replay is unchanged
    s2 = Snap(data)
    s2.clock = 101
    data2 = s2.close()
    assert data2 == data and replay(data2) == (0, {FOO}, [100, 42, 50])


def test_snapshoter_force_compact_kat():
    """snapshoter_force_compact: min compact size 1024, events and queries with ltime
    0..1023; the log compacts and still replays to 1023 / 1023."""
    s = Snap(min_compact=1024)
    for i in range(1024):
        s.user(i)
    for i in range(1024):
        s.query(i)
    comp = s.sp.compactions
    data = s.close()
    rc, alive, clocks = replay(data)
    assert rc == 0 and clocks[1] == 1023 and clocks[2] == 1023 and alive == set()
    assert comp > 0 and len(data) <= 1024 + 9


@pytest.mark.parametrize("rejoin", [False, True])
def test_snapshoter_leave_kat(rejoin):
    """snapshoter_leave / snapshoter_leave_rejoin: after a leave the replay is empty
    (clocks 0, no alive nodes) unless rejoin_after_leave keeps the state."""
    s = Snap(rejoin=rejoin)
    s.user(42)
    s.query(50)
    s.witness(100)
    s.member(EV_JOIN, FOO)
    s.leave()
    s.user(77)  # recording stopped after the leave
    s.member(EV_JOIN, FOO + 1)
    data = s.close()
    rc, alive, clocks = replay(data, rejoin)
    assert rc == 0
    if rejoin:
        assert clocks == [100, 42, 50] and alive == {FOO}
    else:
        assert clocks == [0, 0, 0] and alive == set()


def test_replay_errors_and_ignored_records():
    clock = bytes([2]) + (5).to_bytes(8, "little")
    assert replay(clock + bytes([5, 7]) + clock)[0] == 0  # Coordinate / Comment are skipped
    assert replay(bytes([9]))[0] == -1                     # UnknownRecordType
    assert replay(bytes([2, 1, 2]))[0] == -2               # truncated clock
    assert replay(bytes([0, 4, 0, 0, 0, 1]))[0] == -2      # truncated node
    assert replay(bytes([0, 2, 0, 0, 0, 1, 0]))[0] == -3   # node that does not decode
    # NotAlive removes, later Alive adds back, Leave clears (without rejoin)
    node = lambda tag, s: bytes([tag, 4, 0, 0, 0]) + s.to_bytes(4, "little")  # noqa: E731
    assert replay(node(0, 3) + node(0, 4) + node(1, 3))[1] == {4}
    assert replay(node(0, 3) + bytes([6]) + node(0, 5))[1] == {5}
    assert replay(node(0, 3) + bytes([6]) + node(0, 5), rejoin=True)[1] == {3, 5}


# ---------------------------------------------------------------- world snapshotters
def _world(n=600, rounds=14, seed=3):
    subj, acts, ml = W.churn_workload(n, rounds, events_per_round=12, queries_per_round=3, seed=seed)
    s = len(subj)
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=16, gossip_limit=400, max_rumors=1 << 14,
                         event_buffer_size=64, query_buffer_size=64, slot_k=8, seed=seed)
    w = H.oracle_world(cfg, subj, W.initial_views(s))
    return w, cfg, subj, acts, ml


def encode(w, m):
    size = L.orc_world_snapshot_encode(C.byref(w), m, None)
    out = np.zeros(max(1, size), np.uint8)
    assert L.orc_world_snapshot_encode(C.byref(w), m, O.ptr(out, C.c_uint8)) == size
    return bytes(out[:size])


def test_world_snapshot_tracks_member_events_and_clocks():
    w, cfg, subj, acts, ml = _world()
    assert L.orc_world_enable_snapshot(C.byref(w), 0) == 0
    n, s = w.n, w.s
    for t in range(len(ml)):
        H.oracle_round(w, t, ml[t], acts[t])
    bits = O.arr(w.snap_bits, n * w.snap_w, np.uint32).reshape(n, w.snap_w)
    sn = O.arr(w.snap_sn, n * 4, np.uint64).reshape(n, 4)
    kind = O.arr(w.v_kind, n * s, np.uint8).reshape(n, s)
    status = O.arr(w.v_status, n * s, np.uint8).reshape(n, s)
    clock = O.arr(w.clock, n, np.uint64)
    changed = 0
    for m in range(0, n, 7):
        rc, alive, clocks = replay(encode(w, m), s=s)
        assert rc == 0
        want = {j for j in range(s) if bits[m, j >> 5] >> (j & 31) & 1}
        assert alive == want
        # live members: the alive set is every Alive / Leaving member the view knows, plus
        # pruned ones (handle_prune emits Reap, which the snapshotter ignores)
        if not sn[m, 3] & 1:
            view = {j for j in range(s) if kind[m, j] == O.K_KNOWN and status[m, j] in (O.ST_ALIVE, O.ST_LEAVING)}
            own = {int(O.arr(w.member_subj, n, np.int32)[m])}
            assert view - own <= alive and all(kind[m, j] == O.K_UNKNOWN for j in alive - view - own)
            assert clocks == [int(clock[m]) - 1, int(sn[m, 0]), int(sn[m, 1])]
        changed += sn[m, 0] > 0
    assert changed > 0
    L.orc_world_free(C.byref(w))


def test_world_restart_from_snapshot():
    """serf_snapshot_recovery in the round model: a member restarts from its own
    snapshot file, its clocks witness the replayed ones, and a user event older than
    the snapshot is not delivered again; it rejoins and learns every live member."""
    w, cfg, subj, acts, ml = _world(seed=4)
    assert L.orc_world_enable_snapshot(C.byref(w), 0) == 0
    n, s = w.n, w.s
    for t in range(8):
        H.oracle_round(w, t, ml[t], acts[t])
    ecl = O.arr(w.eclock, n, np.uint64)
    sn = O.arr(w.snap_sn, n * 4, np.uint64).reshape(n, 4)
    alive = O.arr(w.alive, n, np.uint8)
    m = int(next(i for i in range(n) if alive[i] and sn[i, 0] > 3 and O.arr(w.member_subj, n, np.int32)[i] < 0))
    data = encode(w, m)
    old_e, old_c = int(sn[m, 0]), int(O.arr(w.clock, n, np.uint64)[m]) - 1
    a = u8(data)
    assert L.orc_world_restart(C.byref(w), m, O.ptr(a, C.c_uint8), len(data)) == 1  # rejoined
    assert int(O.arr(w.clock, n, np.uint64)[m]) == old_c + 1
    assert int(ecl[m]) == old_e + 1 and int(O.arr(w.emin, n, np.uint64)[m]) == old_e + 1
    assert L.orc_handle_user_event(C.byref(w), m, old_e, 0xABCDEF) == 0  # old: not delivered again
    assert L.orc_handle_user_event(C.byref(w), m, old_e + 1, 0xABCDEF) != 0
    kind = O.arr(w.v_kind, n * s, np.uint8).reshape(n, s)
    sm = O.arr(w.subj_member, s, np.uint32)
    up = {j for j in range(s) if alive[sm[j]]}
    assert {j for j in range(s) if kind[m, j] == O.K_KNOWN} == up
    # the rest of the run stays consistent (threaded = sequential after a restart)
    for t in range(8, len(ml)):
        H.oracle_round(w, t, ml[t], acts[t])
    L.orc_world_free(C.byref(w))


def test_node_update_emits_update_event_for_known_members():
    """handle_node_update (base.rs:1532-1583): only a member with state gets the Update
    event; the view is unchanged."""
    w, cfg, subj, acts, ml = _world(rounds=1)
    n, s = w.n, w.s
    dig = O.arr(w.digest, n, np.uint64)
    kind = O.arr(w.v_kind, n * s, np.uint8).reshape(n, s)
    kind[3, 1] = O.K_UNKNOWN
    d0 = int(dig[3])
    assert L.orc_handle_node_update(C.byref(w), 3, 1) == 0 and int(dig[3]) == d0
    view0 = kind.copy()
    assert L.orc_handle_node_update(C.byref(w), 3, 2) == O.F_MEMBER_EVENT and int(dig[3]) != d0
    assert np.array_equal(kind, view0)
    L.orc_world_free(C.byref(w))


def test_reconnect_targets_failed_members_only():
    w, cfg, subj, acts, ml = _world(n=800, rounds=10, seed=6)
    n, s = w.n, w.s
    for t in range(len(ml)):
        H.oracle_round(w, t, ml[t], acts[t])
    kind = O.arr(w.v_kind, n * s, np.uint8).reshape(n, s).copy()
    status = O.arr(w.v_status, n * s, np.uint8).reshape(n, s).copy()
    sm = O.arr(w.subj_member, s, np.uint32)
    alive = O.arr(w.alive, n, np.uint8).copy()
    tgt = np.zeros(n, np.uint32)
    joins = L.orc_world_reconnect(C.byref(w), 3, O.ptr(tgt, C.c_uint32))
    tried = np.nonzero(tgt != 0xFFFFFFFF)[0]
    assert len(tried) > 0
    for m in tried:
        j = int(tgt[m])
        assert alive[m] and kind[m, j] == O.K_KNOWN and status[m, j] == O.ST_FAILED
    ok = [m for m in tried if alive[sm[tgt[m]]]]
    assert joins == len(ok)
    st_after = O.arr(w.v_status, n * s, np.uint8).reshape(n, s)
    for m in ok:
        assert st_after[m, tgt[m]] == O.ST_ALIVE
    # the throttle: members with no failed peers never try
    nf = ((kind == O.K_KNOWN) & (status == O.ST_FAILED)).sum(1)
    assert np.all(tgt[nf == 0] == 0xFFFFFFFF)
    L.orc_world_free(C.byref(w))


def test_reconnect_probability_formula_hand_worked():
    """base.rs:670-671: num_alive = (members.states.len() - num_failed - left_members.len()).max(1),
    prob = num_failed as f32 / num_alive as f32.  At configs[1]'s shape (N = 1M members, S = 4096
    tracked subjects) a member that is not a subject knows the N - S untracked members
    (implicitly Alive, itself among them) plus the tracked subjects it knows: with all 4096
    known, 10 failed and 5 left, states.len() = 1_000_000 and prob = 10 / 999_985."""
    n, s = 1_000_000, 4096
    states = (n - s) + s
    got = L.orc_reconnect_prob(states, 10, 5)
    assert np.float32(got) == np.float32(10) / np.float32(999_985)
    assert abs(got - 1.0000150e-5) < 1e-11
    # the subject itself is not one of the N - S: it adds itself (known = N - S + 1 + tracked others)
    assert np.float32(L.orc_reconnect_prob((n - s) + 1 + 4095, 3, 0)) == np.float32(3) / np.float32(n - 3)
    # .max(1): every known member failed or left
    assert L.orc_reconnect_prob(7, 4, 3) == 4.0
    # the tracked-only count (round-2 model) would be ~244x larger at this shape
    assert L.orc_reconnect_prob(s + 1, 10, 5) / got > 240


def test_reconnect_throttle_uses_states_len():
    """The world's Reconnector draws each member's throttle exactly as the formula above with
    states.len() = (n - s) + [member is a subject] + its KNOWN tracked subjects, and the same
    Philox draw (purpose 7, counter (0, 7 << 24, member, tick))."""
    w, cfg, subj, acts, ml = _world(n=800, rounds=10, seed=6)
    n, s = w.n, w.s
    for t in range(len(ml)):
        H.oracle_round(w, t, ml[t], acts[t])
    kind = O.arr(w.v_kind, n * s, np.uint8).reshape(n, s).copy()
    status = O.arr(w.v_status, n * s, np.uint8).reshape(n, s).copy()
    msubj = O.arr(w.member_subj, n, np.int32).copy()
    alive = O.arr(w.alive, n, np.uint8).copy()
    seed = cfg.seed
    key = np.array([seed & 0xFFFFFFFF, seed >> 32], np.uint32)
    tick = 5
    expect_try = np.zeros(n, bool)
    for m in range(n):
        if not alive[m]:
            continue
        own = int(msubj[m])
        mask = np.ones(s, bool)
        if own >= 0:
            mask[own] = False
        kn = mask & (kind[m] == O.K_KNOWN)
        failed = int((kn & (status[m] == O.ST_FAILED)).sum())
        left = int((kn & (status[m] == O.ST_LEFT)).sum())
        if failed == 0:
            continue
        states = (n - s) + (1 if own >= 0 else 0) + int(kn.sum())
        prob = np.float32(failed) / np.float32(max(states - failed - left, 1))
        ctr = np.array([0, 7 << 24, m, tick], np.uint32)
        out = np.zeros(4, np.uint32)
        L.orc_philox4x32(O.ptr(ctr, C.c_uint32), O.ptr(key, C.c_uint32), O.ptr(out, C.c_uint32))
        r = np.float32(int(out[0]) >> 8) * np.float32(1.0 / 16777216.0)
        expect_try[m] = not (r > prob)
    tgt = np.zeros(n, np.uint32)
    L.orc_world_reconnect(C.byref(w), tick, O.ptr(tgt, C.c_uint32))
    assert np.array_equal(tgt != 0xFFFFFFFF, expect_try)
    L.orc_world_free(C.byref(w))
