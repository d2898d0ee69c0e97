"""Pins the CPU oracle (oracle/oracle.c) against the known answers held by
al8n/ruserf's own unit tests (tests/golden/reference_kats.json, transcribed
from the cited reference file:line).  CPU only."""
import ctypes as C
import math

import numpy as np
import pytest

import oracle_ffi as O

L = O.lib()


def test_philox_random123_kat():
    # Random123 kat_vectors for philox4x32_10 (the counter-based RNG the build
    # uses in place of the reference's thread_rng)
    cases = [
        ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
        ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
        ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
         (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
    ]
    for ctr, key, exp in cases:
        c = (C.c_uint32 * 4)(*ctr)
        k = (C.c_uint32 * 2)(*key)
        o = (C.c_uint32 * 4)()
        L.orc_philox4x32(c, k, o)
        assert tuple(o) == exp


# ---------------------------------------------------------------- Vivaldi
def test_opts_default(kats):
    d = kats["coordinate"]["opts_default"]
    o = O.default_opts()
    for k in ["dimensionality", "vivaldi_error_max", "vivaldi_ce", "vivaldi_cc",
              "adjustment_window_size", "height_min", "latency_filter_size", "gravity_rho"]:
        assert getattr(o, k) == d[k], k


def _client(opts, slots=4):
    c = O.Client()
    assert L.orc_client_init(C.byref(c), C.byref(opts), slots) == 0
    return c


def test_client_update(kats):
    k = kats["coordinate"]["client_update"]
    opts = O.default_opts(dimensionality=k["dim"])
    cl = _client(opts)
    assert list(cl.coord.portion[:3]) == [0.0, 0.0, 0.0]
    other = O.coord(opts, k["other_portion"])
    out = O.Coord()
    r = O.rng()
    assert L.orc_client_update(C.byref(cl), 0, C.byref(other), k["rtt_ns"], C.byref(r), C.byref(out)) == O.OK
    assert out.portion[2] < 0.0
    out.portion[2] = 99.0
    assert L.orc_client_set_coordinate(C.byref(cl), C.byref(out)) == O.OK
    assert cl.coord.portion[2] == 99.0
    L.orc_client_free(C.byref(cl))


def test_client_invalid_in_ping_values(kats):
    k = kats["coordinate"]["client_invalid_in_ping_values"]
    opts = O.default_opts(dimensionality=k["dim"])
    cl = _client(opts)
    other = O.coord(opts, k["other_portion"])
    dist = L.orc_coord_distance_ns(C.byref(cl.coord), C.byref(other))
    for ns in k["rtt_ns"]:
        r = O.rng()
        assert L.orc_client_update(C.byref(cl), 0, C.byref(other), ns, C.byref(r), None) == O.ERR_RTT
        assert L.orc_coord_distance_ns(C.byref(cl.coord), C.byref(other)) == dist
    L.orc_client_free(C.byref(cl))


def test_client_distance_to(kats):
    k = kats["coordinate"]["client_distance_to"]
    opts = O.default_opts(dimensionality=k["dim"], height_min=k["height_min"])
    cl = _client(opts)
    other = O.coord(opts, k["other_portion"])
    assert L.orc_coord_distance_ns(C.byref(cl.coord), C.byref(other)) == k["expect_ns"]
    L.orc_client_free(C.byref(cl))


def test_client_latency_filter(kats):
    k = kats["coordinate"]["client_latency_filter"]
    opts = O.default_opts(latency_filter_size=k["filter_size"])
    cl = _client(opts, slots=2)
    slot = {"alice": 0, "bob": 1}
    for step in k["steps"]:
        if step[0] == "forget":
            L.orc_client_forget_node(C.byref(cl), slot[step[1]])
            continue
        got = L.orc_client_latency_filter(C.byref(cl), slot[step[0]], step[1])
        assert got == step[2]  # the reference checks |d| <= 1e-6; the median is exact
    L.orc_client_free(C.byref(cl))


def test_client_nan_defense(kats):
    k = kats["coordinate"]["client_nan_defense"]
    opts = O.default_opts(dimensionality=k["dim"])
    cl = _client(opts)
    other = O.coord(opts, [math.nan, 0.0, 0.0])
    assert not L.orc_coord_is_valid(C.byref(other))
    r = O.rng()
    assert L.orc_client_update(C.byref(cl), 0, C.byref(other), k["rtt_ns"], C.byref(r), None) == O.ERR_COORD
    assert L.orc_coord_is_valid(C.byref(cl.coord))
    wide = O.coord(opts, [math.nan, 0.0, 0.0, 0.0, 0.0, 0.0])
    assert L.orc_client_set_coordinate(C.byref(cl), C.byref(wide)) == O.ERR_DIM
    assert L.orc_coord_is_valid(C.byref(cl.coord))
    cl.coord.portion[0] = math.nan
    good = O.coord(opts)
    out = O.Coord()
    assert L.orc_client_update(C.byref(cl), 0, C.byref(good), k["rtt_ns"], C.byref(r), C.byref(out)) == O.OK
    assert L.orc_coord_is_valid(C.byref(out))
    assert cl.resets == 1
    L.orc_client_free(C.byref(cl))


def test_coordinate_apply_force(kats):
    k = kats["coordinate"]["coordinate_apply_force"]
    for case in k["cases"]:
        opts = O.default_opts(dimensionality=k["dim"], height_min=case["height_min"])
        me = O.coord(opts, case["self"], height=case["self_height"])
        other = O.coord(opts, case["other"], height=case["other_height"])
        r = O.rng()
        L.orc_apply_force_in_place(C.byref(me), case["height_min"], case["force"], C.byref(other), C.byref(r))
        for i in range(3):
            assert abs(me.portion[i] - case["expect_portion"][i]) <= 1e-6
            # exact where the arithmetic is exact
        if "expect_height" in case:
            assert abs(me.height - case["expect_height"]) <= 1e-6
    rc = k["random_case"]
    opts = O.default_opts(dimensionality=k["dim"], height_min=rc["height_min"])
    origin = O.coord(opts)
    me = O.coord(opts)
    r = O.rng(member=7)
    L.orc_apply_force_in_place(C.byref(me), rc["height_min"], rc["force"], C.byref(origin), C.byref(r))
    d = L.orc_as_secs_f64(L.orc_coord_distance_ns(C.byref(origin), C.byref(me)))
    assert abs(d - rc["expect_distance_secs"]) <= 1e-6


def test_vector_helpers(kats):
    k = kats["coordinate"]
    v = (C.c_double * 3)(*k["coordinate_magnitude"]["v"])
    assert L.orc_magnitude(v, 3) == k["coordinate_magnitude"]["expect"]
    z = (C.c_double * 3)(0.0, 0.0, 0.0)
    assert L.orc_magnitude(z, 3) == 0.0
    u = k["coordinate_unit_vector_at"]
    a = (C.c_double * 3)(*u["a"])
    b = (C.c_double * 3)(*u["b"])
    out = (C.c_double * 3)()
    r = O.rng()
    mag = L.orc_unit_vector_at(a, b, 3, out, C.byref(r))
    for i in range(3):
        assert abs(out[i] - u["expect"][i]) <= 1e-15
    d = (C.c_double * 3)(*[x - y for x, y in zip(u["a"], u["b"])])
    assert mag == L.orc_magnitude(d, 3)
    assert abs(L.orc_magnitude(out, 3) - 1.0) <= 1e-6
    mag = L.orc_unit_vector_at(a, a, 3, out, C.byref(r))
    assert mag == 0.0 and abs(L.orc_magnitude(out, 3) - 1.0) <= 1e-6
    # add / diff (coordinate.rs:1160-1197) are elementwise IEEE ops
    ad, df = k["coordinate_add"], k["coordinate_diff"]
    assert [x + y for x, y in zip(ad["a"], ad["b"])] == ad["expect"]
    assert [x - y for x, y in zip(df["a"], df["b"])] == df["expect"]


def test_as_secs_f64_and_saturating_cast():
    # Duration::as_secs_f64 is secs + nanos/1e9, which differs from ns/1e9
    diffs = 0
    for ns in range(1_000_000_007, 1_000_000_007 + 20000 * 7919, 7919):
        a = L.orc_as_secs_f64(ns)
        assert a == (ns // 10**9) + (ns % 10**9) / 1e9
        diffs += a != ns / 1e9
    assert diffs > 0
    opts = O.default_opts(dimensionality=3, height_min=0.0)
    a = O.coord(opts)
    b = O.coord(opts, [0.0, 0.0, 1e300])
    assert L.orc_coord_distance_ns(C.byref(a), C.byref(b)) == 2**64 - 1


# ------------------------------------------------------------ Lamport clock
def test_lamport_clock(kats):
    # LamportClock::{time, increment, witness} restated in oracle.h
    clock = 0
    for op in kats["clock"]["ops"]:
        if op[0] == "time":
            assert clock == op[1]
        elif op[0] == "increment":
            clock += 1
            assert clock == op[1]
        else:
            if not op[1] < clock:
                clock = op[1] + 1
            assert clock == op[2]


# ---------------------------------------------------------------- merge
def make_world(n=2, s=1, **kw):
    cfg = O.WorldCfg(n=n, s=s, qcap=8, ebuf=512, qbuf=512, slot_k=8, fanout=1, limit=1400,
                     overhead=2, retransmit_mult=4, max_refute=2, cap_rumors=1024, seed=0x5EED5EED)
    for k_, v in kw.items():
        setattr(cfg, k_, v)
    w = O.World()
    assert L.orc_world_init(C.byref(w), C.byref(cfg)) == 0
    for i in range(s):
        w.subj_member[i] = n - s + i
        w.member_subj[n - s + i] = i
    return w


def set_known(w, m, subj, status, st):
    e = m * w.s + subj
    w.v_kind[e] = O.K_KNOWN
    w.v_status[e] = status
    w.v_ltime[e] = st


def intent(w, m, subj):
    e = m * w.s + subj
    return {O.K_JOIN: "join", O.K_LEAVE: "leave"}.get(w.v_kind[e]), w.v_ltime[e]


STATUS = {"alive": O.ST_ALIVE, "leaving": O.ST_LEAVING, "left": O.ST_LEFT, "failed": O.ST_FAILED}


@pytest.mark.parametrize("name", ["join_intent_buffer_early", "leave_intent_buffer_early"])
def test_intent_buffer_early(kats, name):
    k = kats["merge"][name]
    w = make_world()
    fn = (lambda: L.orc_handle_join_intent(C.byref(w), 0, 0, k["ltime"])) if name.startswith("join") \
        else (lambda: L.orc_handle_leave_intent(C.byref(w), 0, 0, k["ltime"], 0, None))
    assert [bool(fn() & O.F_REBROADCAST) for _ in range(2)] == k["expect"]
    assert list(intent(w, 0, 0)) == k["buffered"]
    L.orc_world_free(C.byref(w))


@pytest.mark.parametrize("name", ["join_intent_old_message", "leave_intent_old_message"])
def test_intent_old_message(kats, name):
    k = kats["merge"][name]
    w = make_world()
    set_known(w, 0, 0, STATUS[k["subject"][0]], k["subject"][1])
    if name.startswith("join"):
        f = L.orc_handle_join_intent(C.byref(w), 0, 0, k["ltime"])
    else:
        f = L.orc_handle_leave_intent(C.byref(w), 0, 0, k["ltime"], 0, None)
    assert bool(f & O.F_REBROADCAST) == k["expect"]
    assert w.v_kind[0] == O.K_KNOWN  # nothing buffered
    L.orc_world_free(C.byref(w))


def test_join_intent_newer_and_reset_leaving(kats):
    for name in ["join_intent_newer", "join_intent_reset_leaving"]:
        k = kats["merge"][name]
        w = make_world()
        set_known(w, 0, 0, STATUS[k["subject"][0]], k["subject"][1])
        assert bool(L.orc_handle_join_intent(C.byref(w), 0, 0, k["ltime"]) & O.F_REBROADCAST) == k["expect"]
        assert w.v_ltime[0] == k["status_time"]
        assert w.clock[0] == k["clock"]
        if "status" in k:
            assert w.v_status[0] == STATUS[k["status"]]
        L.orc_world_free(C.byref(w))


def test_leave_intent_newer(kats):
    k = kats["merge"]["leave_intent_newer"]
    w = make_world()
    set_known(w, 0, 0, O.ST_ALIVE, 12)
    assert bool(L.orc_handle_leave_intent(C.byref(w), 0, 0, k["ltime"], 0, None) & O.F_REBROADCAST)
    assert w.v_status[0] == STATUS[k["status"]]
    assert w.clock[0] == k["clock"]
    L.orc_world_free(C.byref(w))


def test_join_pending_intents(kats):
    for name in ["join_pending_intent", "join_pending_intents"]:
        k = kats["merge"][name]
        w = make_world()
        for ty, lt in k["intents"]:
            L.orc_upsert_intent(C.byref(w), 0, 0, O.K_JOIN if ty == "join" else O.K_LEAVE, lt)
        L.orc_handle_node_join(C.byref(w), 0, 0)
        assert w.v_kind[0] == O.K_KNOWN
        assert w.v_status[0] == STATUS[k["after_node_join"][0]]
        assert w.v_ltime[0] == k["after_node_join"][1]
        L.orc_world_free(C.byref(w))


def test_leave_transitions_and_refute():
    # base.rs:1466-1527 state table, plus the self-refute branch (1437-1447)
    w = make_world(n=3, s=1)
    for st, exp_st, exp_flags in [
        (O.ST_ALIVE, O.ST_LEAVING, O.F_REBROADCAST),
        (O.ST_LEAVING, O.ST_LEAVING, O.F_REBROADCAST),
        (O.ST_LEFT, O.ST_LEFT, O.F_REBROADCAST),
        (O.ST_FAILED, O.ST_LEFT, O.F_REBROADCAST | O.F_MEMBER_EVENT),
        (O.ST_NONE, O.ST_NONE, 0),
    ]:
        set_known(w, 0, 0, st, 5)
        f = L.orc_handle_leave_intent(C.byref(w), 0, 0, 9, 0, None)
        assert f == exp_flags and w.v_status[0] == exp_st and w.v_ltime[0] == 9
    # receiver == subject (member 2) and alive -> refute with clock.time()
    set_known(w, 2, 0, O.ST_ALIVE, 5)
    ref = C.c_uint64(0)
    f = L.orc_handle_leave_intent(C.byref(w), 2, 0, 9, 0, C.byref(ref))
    assert f == O.F_REFUTE and ref.value == w.clock[2] == 10 and w.v_ltime[2 * w.s] == 5
    L.orc_world_free(C.byref(w))


def test_leave_intent_prune():
    """force_leave(prune=true) (api.rs:565 remove_failed_node_prune -> base.rs:474-500)
    -> handle_node_leave_intent -> handle_prune (base.rs:1472-1526, 1587-1612): the
    member is erased from members.states (the reference test serf_remove_failed_node_prune,
    tests/serf/remove.rs:96-164, waits for the survivors to count 2 nodes, i.e. the
    failed member gone), a Reap MemberEvent follows (after the Leave event of a Failed
    member), the message is still rebroadcast; the next intent about the member is
    buffered by upsert_intent as for any unknown member."""
    reap = lambda d, subj: L.orc_digest_mix(d, 0x3000000000000000 | (3 << 32) | subj)  # noqa: E731
    leave = lambda d, subj: L.orc_digest_mix(d, 0x3000000000000000 | (1 << 32) | subj)  # noqa: E731
    for st, flags, events in [
        (O.ST_FAILED, O.F_REBROADCAST | O.F_MEMBER_EVENT | O.F_PRUNE, [leave, reap]),
        (O.ST_ALIVE, O.F_REBROADCAST | O.F_PRUNE, [reap]),
        (O.ST_LEAVING, O.F_REBROADCAST | O.F_PRUNE, [reap]),
        (O.ST_LEFT, O.F_REBROADCAST | O.F_PRUNE, [reap]),
        (O.ST_NONE, 0, []),
    ]:
        w = make_world(n=3, s=1)
        set_known(w, 0, 0, st, 5)
        f = L.orc_handle_leave_intent(C.byref(w), 0, 0, 9, 1, None)
        assert f == flags
        d = 0
        for ev in events:
            d = ev(d, 0)
        assert w.digest[0] == d
        if flags & O.F_PRUNE:
            assert (w.v_kind[0], w.v_status[0], w.v_ltime[0]) == (O.K_UNKNOWN, O.ST_NONE, 0)
            # erased: an older leave intent is now buffered, as for a member never seen
            f2 = L.orc_handle_leave_intent(C.byref(w), 0, 0, 7, 0, None)
            assert f2 == O.F_REBROADCAST and intent(w, 0, 0) == ("leave", 7)
        else:
            assert w.v_kind[0] == O.K_KNOWN and w.v_ltime[0] == 9
        # a stale prune (ltime <= status_time) changes nothing
        w2 = make_world(n=3, s=1)
        set_known(w2, 0, 0, st, 5)
        assert L.orc_handle_leave_intent(C.byref(w2), 0, 0, 5, 1, None) == 0
        assert w2.v_kind[0] == O.K_KNOWN and w2.digest[0] == 0
        L.orc_world_free(C.byref(w))
        L.orc_world_free(C.byref(w2))


def test_queue_prune_counted_and_checker():
    """The bounded queue model drops the last item in send order when full, and
    counts it (RSF_E_QUEUE_PRUNE); QueueChecker (base.rs:703-760) prunes to max."""
    w = make_world(n=2, s=1, qcap=4)
    for i in range(6):
        w.rumors[i].type = 1
        w.rumors[i].msg_len = 20
        L.orc_queue_insert(C.byref(w), 0, 0, i)
    assert w.q_pruned[0] == 2 and w.err[0] & 16
    live = sorted(w.q_rumor[i] for i in range(4))
    assert live == [2, 3, 4, 5]  # same transmits and length: the oldest (smallest seq) go first
    st = (C.c_uint64 * 9)()
    L.orc_check_queues(C.byref(w), 4096, 0, 3, st)
    assert list(st) == [4, 0, 0, 1, 0, 0, 0, 0, 0]
    L.orc_check_queues(C.byref(w), 1, 0, 128, st)  # max 1 -> three dropped, the newest kept
    assert list(st)[6] == 3 and [w.q_rumor[i] for i in range(4) if w.q_rumor[i] != 0xFFFFFFFF] == [5]
    L.orc_world_free(C.byref(w))


def test_checker_phases_compose_to_one_tick():
    """Staggered ticks (orc_check_queues_phase: each node's checker on its own timer,
    base.rs:703-735): the phases 0..p-1 of one period, with nothing in between, are one
    tick over every member -- the same queues kept and the same counts; a phase's tick
    touches only its own members."""
    def world():
        w = make_world(n=7, s=1, qcap=16)
        r = 0
        for m in range(7):
            for i in range(5 + 2 * m):
                w.rumors[r].type = 1
                w.rumors[r].msg_len = 20 + (i % 3)
                L.orc_queue_insert(C.byref(w), m, 0, r)
                r += 1
        return w
    a, b = world(), world()
    full = (C.c_uint64 * 9)()
    L.orc_check_queues(C.byref(a), 6, 0, 8, full)
    tot = np.zeros(9, dtype=np.uint64)
    for ph in range(3):
        before = [b.q_rumor[i] for i in range(7 * 3 * 16)]
        st = (C.c_uint64 * 9)()
        L.orc_check_queues_phase(C.byref(b), 6, 0, 8, 3, ph, st)
        tot += np.array(list(st), dtype=np.uint64)
        for m in range(7):
            if m % 3 != ph:  # other phases' members untouched
                assert [b.q_rumor[i] for i in range(m * 48, m * 48 + 48)] == before[m * 48:m * 48 + 48]
    assert list(tot) == list(full)
    assert [a.q_rumor[i] for i in range(7 * 3 * 16)] == [b.q_rumor[i] for i in range(7 * 3 * 16)]
    assert int(full[6]) == sum(max(0, min(5 + 2 * m, 16) - 6) for m in range(7))  # (16 slots: one dropped on insert)
    L.orc_world_free(C.byref(a))
    L.orc_world_free(C.byref(b))


def test_queue_depth_per_queue_and_checker():
    """Per-queue capacities (orc_world_cfg.qdepth, the engine's queue_depth): each queue
    prunes at its own depth, slots past it stay unused, scans stop at the high-water mark,
    and the QueueChecker counts and prunes head-and-tail queues the same way."""
    cfg = O.WorldCfg(n=2, s=1, qcap=16, ebuf=512, qbuf=512, slot_k=8, fanout=1, limit=1400, overhead=2,
                     retransmit_mult=4, max_refute=2, cap_rumors=1024, seed=0x5EED5EED)
    cfg.qdepth[:] = [4, 16, 8]
    w = O.World()
    assert L.orc_world_init(C.byref(w), C.byref(cfg)) == 0
    assert list(w.qd) == [4, 16, 8]
    for i in range(30):
        w.rumors[i].type = 1
        w.rumors[i].msg_len = 20
    for q in range(3):
        for i in range(10):
            L.orc_queue_insert(C.byref(w), 0, q, 10 * q + i)
    live = [[w.q_rumor[q * 16 + i] for i in range(16) if w.q_rumor[q * 16 + i] != 0xFFFFFFFF] for q in range(3)]
    assert sorted(live[0]) == [6, 7, 8, 9]            # depth 4: the newest four kept
    assert sorted(live[1]) == list(range(10, 20))     # depth 16: nothing dropped
    assert sorted(live[2]) == list(range(22, 30))     # depth 8
    assert w.q_pruned[0] == 6 + 2
    assert [w.q_hwm[q] for q in range(3)] == [4, 10, 8]
    # a pick frees a slot below the high-water mark; the next insert reuses it
    out, used = (C.c_uint32 * 8)(), C.c_uint32()
    w.tx_limit = 1  # every pick retires
    assert L.orc_queue_get_broadcasts(C.byref(w), 0, 1, 22, out, 8, C.byref(used)) == 1
    L.orc_queue_insert(C.byref(w), 0, 1, 29)
    assert w.q_hwm[1] == 10
    st = (C.c_uint64 * 9)()
    L.orc_check_queues(C.byref(w), 5, 0, 8, st)
    assert list(st) == [4, 10, 8, 0, 1, 1, 0, 5, 3]
    L.orc_world_free(C.byref(w))


def test_delegate_merge_remote_state(kats):
    """merge_remote_state (delegate.rs:422-554) through orc_merge_remote_state: the
    reference test's PushPullMessage becomes a sender local_state (status_ltimes ->
    KNOWN entries, left_members -> status Left, the event buffer slot 45)."""
    k = kats["merge"]["delegate_merge_remote_state"]
    pp = k["pp"]
    # subjects: test=0, foo=1; receiver = member 0
    w = make_world(n=3, s=2)
    subj = {"test": 0, "foo": 1}
    names = {"test": 1}
    v_lt = np.zeros(2, np.uint64)
    v_st = np.zeros(2, np.uint8)
    v_kd = np.zeros(2, np.uint8)
    for node, lt in pp["status_ltimes"]:
        v_lt[subj[node]] = lt
        v_kd[subj[node]] = O.K_KNOWN
        v_st[subj[node]] = O.ST_LEFT if node in pp["left_members"] else O.ST_ALIVE
    eb_lt = np.zeros(w.ebuf, np.uint64)
    eb_cnt = np.zeros(w.ebuf, np.uint32)
    eb_keys = np.zeros(w.ebuf * w.slot_k, np.uint64)
    for ltime, evs in pp["events"]:
        slot = ltime % w.ebuf
        eb_lt[slot] = ltime
        for name, _payload in evs:
            eb_keys[slot * w.slot_k + eb_cnt[slot]] = names[name] << 32
            eb_cnt[slot] += 1
    st = O.PPState(pp["ltime"], pp["event_ltime"], pp["query_ltime"], O.ptr(v_lt, C.c_uint64),
                   O.ptr(v_st, C.c_uint8), O.ptr(v_kd, C.c_uint8), O.ptr(eb_lt, C.c_uint64),
                   O.ptr(eb_cnt, C.c_uint32), O.ptr(eb_keys, C.c_uint64))
    assert L.orc_merge_remote_state(C.byref(w), 0, C.byref(st), 0, 0) == 0
    e = k["expect"]
    assert w.clock[0] == e["clock"]
    assert list(intent(w, 0, 0)) == e["intent_test"]
    assert list(intent(w, 0, 1)) == e["intent_foo"]
    assert w.eclock[0] == e["event_clock"]
    assert w.eb_cnt[45] == 1 and w.eb_keys[45 * w.slot_k] >> 32 == names[e["event_slot_45_name"]]
    assert w.qclock[0] == e["query_clock"]
    L.orc_world_free(C.byref(w))


# ---------------------------------------------------------- dissemination
def test_user_event_old_message(kats):
    k = kats["dissemination"]["user_event_old_message"]
    w = make_world()
    if not k["witness"] < w.eclock[0]:
        w.eclock[0] = k["witness"] + 1
    assert L.orc_handle_user_event(C.byref(w), 0, k["ltime"], 7) == 0
    L.orc_world_free(C.byref(w))


def test_user_event_same_clock(kats):
    k = kats["dissemination"]["user_event_same_clock"]
    w = make_world()
    names, payloads = {}, {}
    keys = []
    for lt, name, payload in k["events"]:
        key = (names.setdefault(name, len(names) + 1) << 32) | payloads.setdefault(payload, len(payloads) + 1)
        keys.append(key)
        f = L.orc_handle_user_event(C.byref(w), 0, lt, key)
        assert bool(f & O.F_REBROADCAST)
        assert bool(f & O.F_DELIVER)
    slot = 1 % 512
    assert [w.eb_keys[slot * w.slot_k + i] for i in range(w.eb_cnt[slot])] == keys
    # a repeat of an already-buffered (name, payload) is not delivered again
    assert L.orc_handle_user_event(C.byref(w), 0, 1, keys[1]) == 0
    L.orc_world_free(C.byref(w))


def test_query_old_message_quirk(kats):
    k = kats["dissemination"]["query_old_message"]
    w = make_world()
    if not k["witness"] < w.qclock[0]:
        w.qclock[0] = k["witness"] + 1
    assert L.orc_handle_query(C.byref(w), 0, k["ltime"], k["id"], 0) == 0
    # quirk (base.rs:999): compares the buffer length, so even a CURRENT query is
    # dropped once the clock exceeds 2*buffer
    assert L.orc_handle_query(C.byref(w), 0, w.qclock[0], 99, 0) == 0
    L.orc_world_free(C.byref(w))


def test_query_same_clock(kats):
    k = kats["dissemination"]["query_same_clock"]
    w = make_world()
    got = [bool(L.orc_handle_query(C.byref(w), 0, lt, qid, 0) & O.F_REBROADCAST) for lt, qid, _ in k["queries"]]
    assert got == k["expect"]
    slot = 1
    assert [w.qb_ids[slot * w.slot_k + i] for i in range(w.qb_cnt[slot])] == [1, 2, 3]
    L.orc_world_free(C.byref(w))


def test_user_event_coalesce_basic(kats):
    k = kats["dissemination"]["user_event_coalesce_basic"]
    names, payloads = {}, {"": 0}
    ev = (O.UEvent * len(k["events"]))()
    for i, (name, lt, payload) in enumerate(k["events"]):
        ev[i].name = names.setdefault(name, len(names) + 1)
        ev[i].ltime = lt
        ev[i].payload = payloads.setdefault(payload, len(payloads))
    out = (O.UEvent * len(k["events"]))()
    n = L.orc_coalesce_user_events(ev, len(k["events"]), out)
    inv_n = {v: kk for kk, v in names.items()}
    inv_p = {v: kk for kk, v in payloads.items()}
    got = [[inv_n[out[i].name], out[i].ltime, inv_p[out[i].payload]] for i in range(n)]
    assert got == k["expect_flushed"]


def test_retransmit_limit():
    # memberlist retransmitLimit = mult * ceil(log10(n+1)) (parity unpinned)
    for n, exp in [(1, 4), (9, 4), (10, 8), (99, 8), (100, 12), (1_000_000, 28), (999_999, 24)]:
        assert L.orc_retransmit_limit(4, n) == exp


def test_serf_reap_handler(kats):
    """Reaper tick (reap.rs:41-131): left members older than tombstone_timeout and
    intents older than recent_intent_timeout go, the rest stay.  Each reference
    left_members entry is its own subject here; time unit = seconds, now = 100."""
    k = kats["merge"]["serf_reap_handler"]
    ages, intents = k["left_ages_s"], k["intents"]
    s = len(ages) + len(intents)
    w = make_world(n=s + 2, s=s)
    now = 100
    for i, age in enumerate(ages):
        set_known(w, 0, i, O.ST_LEFT, 0)
        w.v_time[i] = now - age
    for j, (_node, ty, lt, age) in enumerate(intents):
        w.now = now - age
        assert L.orc_upsert_intent(C.byref(w), 0, len(ages) + j, O.K_JOIN if ty == "join" else O.K_LEAVE, lt) == 1
    d0 = w.digest[0]
    L.orc_reap(C.byref(w), now, 1 << 30, k["tombstone_timeout_s"], k["recent_intent_timeout_s"])
    left = [w.v_kind[i] == O.K_KNOWN and w.v_status[i] == O.ST_LEFT for i in range(len(ages))]
    assert sum(left) == k["expect_left_remaining"]
    kept = [node for j, (node, *_r) in enumerate(intents) if w.v_kind[len(ages) + j] != O.K_UNKNOWN]
    assert kept == k["expect_intents_kept"]
    assert w.digest[0] != d0  # one Reap member event was emitted
    L.orc_world_free(C.byref(w))


def test_configs0_c1_converges_on_cpu():
    """BASELINE configs[0] on the CPU path: 1000 clients x 1000 rounds of the
    oracle's CoordinateClient::update over the synthetic 1k-node RTT matrix; the final median
    |estimate_rtt - true| / true over all pairs is small (~5%), and no coordinate reset."""
    import bench
    r = bench.c1_leg(with_gpu=False)
    assert r["median_rel_rtt_error_all_pairs"] < 0.1
    assert r["resets"] == 0 and r["cpu_updates_per_s"] > 0


# ---------------------------------------------------------------- origination size limits
def _round_with(w, act, name_len, payload_len, t=0):
    a = (O.Action * 1)()
    a[0].member, a[0].act, a[0].name_len, a[0].payload_len, a[0].key = 0, act, name_len, payload_len, 7
    assert L.orc_world_round(C.byref(w), t, None, 0, a, 1) == 0
    st = (C.c_int32 * 1)()
    assert L.orc_world_action_status(C.byref(w), st, 1) == 0
    return st[0]


def test_origination_size_limit_kats(kats):
    """The reference's size-limit tests against the oracle's restatement of Serf::user_event
    (api.rs:255-287) and query_in (base.rs:916-921): serf_event_user_size_limit
    (event.rs:506-525), serf_query_size_limit (:1070-1085) and _increased (:1087-1100).
    A rejected origination moves no clock and queues nothing."""
    d = kats["dissemination"]
    ue_lim, q_lim = d["max_user_event_size"]["value"], d["query_size_limit"]["value"]
    assert d["user_event_size_limit_const"]["value"] == 9216
    k = d["serf_event_user_size_limit"]
    assert L.orc_user_event_check(ue_lim, 1, len(k["name"]), ue_lim) == -20  # UserEventLimitTooLarge
    assert L.orc_user_event_check(ue_lim, 1, len(k["name"]), ue_lim - len(k["name"])) == -22  # encoded > limit
    assert L.orc_user_event_check(ue_lim, 1, 8, 32) == 0
    # the sane limit only binds through the encoded length when the option sits at 9 KiB
    assert L.orc_user_event_check(9216, 1, 9216 - 8, 8) == -22
    assert L.orc_user_event_check(9216, 1, 9216, 1) == -20
    kq = d["serf_query_size_limit"]
    assert L.orc_query_check(q_lim * kq["query_size_limit_factor"], 1, len(kq["name"]), q_lim) == -23
    kq2 = d["serf_query_size_limit_increased"]
    assert L.orc_query_check(q_lim * kq2["query_size_limit_factor"], 1, len(kq2["name"]), q_lim) == 0
    # the encoded length depends on the clock's varint width: 127 -> 1 byte, 128 -> 2
    base = L.orc_msg_len(4, 127, 0, 0) - 1  # RSF_MSG_QUERY
    assert L.orc_query_check(base, 127, 0, 0) == 0 and L.orc_query_check(base, 128, 0, 0) == -23

    # through a round: nothing moves for a rejected event / query, the accepted ones queue
    w = make_world(n=4, s=1)
    e0, q0, c0 = w.eclock[0], w.qclock[0], w.clock[0]
    assert _round_with(w, O.ACT_USER_EVENT, len(k["name"]), ue_lim) == -20
    assert (w.eclock[0], w.qclock[0], w.clock[0]) == (e0, q0, c0)
    assert all(w.q_next_seq[i] == 0 for i in range(12)) and all(w.digest[m] == 0 for m in range(4))
    assert _round_with(w, O.ACT_QUERY, len(kq["name"]), q_lim, t=1) == -23
    assert all(w.q_next_seq[i] == 0 for i in range(12))
    L.orc_world_free(C.byref(w))
    w = make_world(n=4, s=1, query_size_limit=2 * q_lim)
    assert _round_with(w, O.ACT_QUERY, len(kq2["name"]), q_lim) == 0
    assert w.q_next_seq[1] == 1  # the origin's query queue took it
    L.orc_world_free(C.byref(w))
    bad = O.WorldCfg(n=2, s=1, qcap=8, ebuf=512, qbuf=512, slot_k=8, fanout=1, limit=1400, overhead=2,
                     retransmit_mult=4, max_refute=2, cap_rumors=1024, max_user_event_size=9217)
    w = O.World()
    assert L.orc_world_init(C.byref(w), C.byref(bad)) == -1  # base.rs:69-70


def test_states_len_and_per_member_queue_max():
    """get_queue_max with min_queue_depth > 0 (base.rs:748-759) reads each node's own
    members.states: 2 * states.len() of that member, so a member that knows fewer tracked
    subjects prunes at a smaller depth."""
    w = make_world(n=6, s=5, qcap=32)
    # member 0 (untracked) knows subjects 0 and 1; member 1 (subject 0) knows nothing else
    set_known(w, 0, 0, O.ST_ALIVE, 1)
    set_known(w, 0, 1, O.ST_LEFT, 1)
    assert L.orc_states_len(C.byref(w), 0) == (6 - 5) + 2
    assert L.orc_states_len(C.byref(w), 1) == (6 - 5) + 1  # itself
    for i in range(40):
        w.rumors[i].type = 1
        w.rumors[i].msg_len = 20
    for m in (0, 1):
        for i in range(20):
            L.orc_queue_insert(C.byref(w), m, 0, 20 * m + i)
    st = (C.c_uint64 * 9)()
    L.orc_check_queues(C.byref(w), 4096, 1, 128, st)
    live = lambda m: sum(w.q_rumor[m * 3 * 32 + i] != 0xFFFFFFFF for i in range(32))  # noqa: E731
    assert (live(0), live(1)) == (6, 4) and st[6] == (20 - 6) + (20 - 4)
    L.orc_world_free(C.byref(w))
