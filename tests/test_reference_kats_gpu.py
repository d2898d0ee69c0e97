"""The reference's own merge / dissemination known answers driven through the GPU engine.

tests/test_oracle_kat.py pins the CPU oracle to these cases; here the same fixtures
(tests/golden/reference_kats.json, transcribed from the reference's direct-handler tests)
go through the HIP engine's C ABI -- rsf_gossip_apply_batch (notify_message),
rsf_gossip_round with a memberlist NotifyJoin / NotifyLeave (handle_node_join / leave),
rsf_gossip_push_pull (merge_remote_state) and rsf_gossip_reap (the Reaper) -- and the
engine's state is asserted against the reference's expected values directly, not against
the oracle:

  join.rs:8-357, leave.rs:4-140        core/src/serf/base/tests/serf/
  event.rs:6-74 (user events), 653-775 (queries)
  delegate.rs:121-186 (push/pull merge_remote_state)
  reap.rs:41-131 (Reaper::run)
"""
import json
import os

import numpy as np
import pytest

from ruserf_amd import gossip as G

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
STATUS = {"alive": G.STATUS_ALIVE, "leaving": G.STATUS_LEAVING, "left": G.STATUS_LEFT, "failed": G.STATUS_FAILED}
INTENT = {G.KIND_INTENT_JOIN: "join", G.KIND_INTENT_LEAVE: "leave"}


@pytest.fixture(scope="module")
def kats():
    with open(os.path.join(HERE, "golden", "reference_kats.json")) as f:
        return json.load(f)


def engine(n=8, s=4, **kw):
    """n members, subjects = the last s members, every subject unknown at every member
    (a fresh Serf that has heard of nobody); the receiver under test is member 0."""
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=8, max_rumors=1024, event_buffer_size=512,
                         query_buffer_size=512, slot_k=8, **kw)
    g = G.GossipEngine(cfg)
    g.set_subjects(np.arange(n - s, n, dtype=np.uint32))
    g.init_views(np.zeros(s, np.uint8), np.zeros(s, np.uint8), np.zeros(s, np.uint64))
    return g


def msgs(rows):
    """(receiver, type, subject, ltime, key, flags) rows -> an rsf_msg batch"""
    m = np.zeros(len(rows), G.MSG_DTYPE)
    for i, (r, t, subj, lt, key, fl) in enumerate(rows):
        m[i]["receiver"], m[i]["type"], m[i]["subject"] = r, t, subj
        m[i]["ltime"], m[i]["key"], m[i]["flags"] = lt, key, fl
    return m


def entry(g, member, subj):
    lt, st, kd, tm = g.view(with_time=True, rows=(member, 1))
    return int(kd[subj]), int(st[subj]), int(lt[subj]), int(tm[subj])


def ml(subject, kind):
    e = np.zeros(1, G.ML_DTYPE)
    e["subject"], e["kind"], e["set_alive"] = subject, kind, 2
    return e


# ------------------------------------------------------------------ merge (join.rs / leave.rs)
@pytest.mark.parametrize("name,mtype", [("join_intent_buffer_early", G.MSG_JOIN),
                                        ("leave_intent_buffer_early", G.MSG_LEAVE)])
def test_intent_buffer_early(kats, name, mtype):
    """An intent about a member not yet known is buffered (upsert_intent) and rebroadcast
    once; the same intent again is not (join.rs:8-35, leave.rs:4-32)."""
    k = kats["merge"][name]
    g = engine()
    flags, _ = g.apply_batch(msgs([(0, mtype, 0, k["ltime"], 0, 0)] * 2))
    assert [bool(f & G.F_REBROADCAST) for f in flags] == k["expect"]
    kd, st, lt, _ = entry(g, 0, 0)
    assert [INTENT[kd], lt] == k["buffered"]
    g.close()


@pytest.mark.parametrize("name,mtype", [("join_intent_old_message", G.MSG_JOIN),
                                        ("leave_intent_old_message", G.MSG_LEAVE)])
def test_intent_old_message(kats, name, mtype):
    """An intent no newer than the known status_time is ignored and nothing is buffered
    (join.rs:38-87, leave.rs:35-84)."""
    k = kats["merge"][name]
    g = engine()
    g.set_view(0, 0, G.KIND_KNOWN, STATUS[k["subject"][0]], k["subject"][1])
    flags, _ = g.apply_batch(msgs([(0, mtype, 0, k["ltime"], 0, 0)]))
    assert bool(flags[0] & G.F_REBROADCAST) == k["expect"]
    kd, st, lt, _ = entry(g, 0, 0)
    assert k["buffered"] is None and kd == G.KIND_KNOWN and lt == k["subject"][1]
    g.close()


@pytest.mark.parametrize("name", ["join_intent_newer", "join_intent_reset_leaving"])
def test_join_intent_newer(kats, name):
    """A newer join intent takes the status_time, witnesses the clock and turns a
    Leaving member back to Alive (join.rs:90-191)."""
    k = kats["merge"][name]
    g = engine()
    g.set_view(0, 0, G.KIND_KNOWN, STATUS[k["subject"][0]], k["subject"][1])
    flags, _ = g.apply_batch(msgs([(0, G.MSG_JOIN, 0, k["ltime"], 0, 0)]))
    assert bool(flags[0] & G.F_REBROADCAST) == k["expect"]
    kd, st, lt, _ = entry(g, 0, 0)
    assert lt == k["status_time"] and int(g.members()["clock"][0]) == k["clock"]
    if "status" in k:
        assert st == STATUS[k["status"]]
    g.close()


def test_leave_intent_newer(kats):
    """A newer leave intent about an Alive member makes it Leaving (leave.rs:87-140)."""
    k = kats["merge"]["leave_intent_newer"]
    g = engine()
    g.set_view(0, 0, G.KIND_KNOWN, STATUS[k["subject"][0]], k["subject"][1])
    flags, _ = g.apply_batch(msgs([(0, G.MSG_LEAVE, 0, k["ltime"], 0, 0)]))
    assert bool(flags[0] & G.F_REBROADCAST) == k["expect"]
    kd, st, lt, _ = entry(g, 0, 0)
    assert st == STATUS[k["status"]] and int(g.members()["clock"][0]) == k["clock"]
    g.close()


@pytest.mark.parametrize("name", ["join_pending_intent", "join_pending_intents"])
def test_join_pending_intents(kats, name):
    """Buffered intents are consumed when memberlist reports the join (handle_node_join):
    a join intent gives Alive at its ltime, a later leave intent Leaving (join.rs:273-357)."""
    k = kats["merge"][name]
    g = engine()
    rows = [(0, G.MSG_JOIN if ty == "join" else G.MSG_LEAVE, 0, lt, 0, 0) for ty, lt in k["intents"]]
    g.apply_batch(msgs(rows))
    g.round(1, ml(0, G.ML_JOIN))  # NotifyJoin about subject 0 at every live member but itself
    kd, st, lt, _ = entry(g, 0, 0)
    assert kd == G.KIND_KNOWN and [st, lt] == [STATUS[k["after_node_join"][0]], k["after_node_join"][1]]
    g.close()


def test_delegate_merge_remote_state(kats):
    """merge_remote_state (delegate.rs:422-554) of the reference test's PushPullMessage
    (delegate.rs:121-186): member 1 holds that local_state (status_ltimes test=20 and foo=15
    with foo left, event buffer slot 45 = "test", clocks 42 / 50 / 100); member 0, which knows
    nobody, merges it.  Expected: clock 42, a buffered join intent test=20, a buffered leave
    intent foo=16, event clock 50, the event in slot 45, query clock 100."""
    k = kats["merge"]["delegate_merge_remote_state"]
    pp, e = k["pp"], k["expect"]
    g = engine(n=4, s=2)
    subj = {"test": 0, "foo": 1}
    names = {"test": 1}
    for node, lt in pp["status_ltimes"]:
        g.set_view(1, subj[node], G.KIND_KNOWN, G.STATUS_LEFT if node in pp["left_members"] else G.STATUS_ALIVE, lt)
    for ltime, evs in pp["events"]:
        for name, _payload in evs:
            g.apply_batch(msgs([(1, G.MSG_USER_EVENT, 0, ltime, names[name] << 32, 0)]))
    g.set_clocks(1, pp["ltime"], pp["event_ltime"], pp["query_ltime"])
    pairs = np.zeros(1, G.PP_PAIR_DTYPE)
    pairs["receiver"], pairs["sender"] = 0, 1
    g.push_pull(pairs)
    m = g.members()
    assert int(m["clock"][0]) == e["clock"]
    assert int(m["event_clock"][0]) == e["event_clock"] and int(m["query_clock"][0]) == e["query_clock"]
    for node, key in [("test", "intent_test"), ("foo", "intent_foo")]:
        kd, st, lt, _ = entry(g, 0, subj[node])
        assert [INTENT.get(kd), lt] == e[key], node
    ebl, ebc, ebk, *_ = g.buffers()
    slot_k = g.cfg.slot_k
    assert ebc[45] == 1 and int(ebk[45 * slot_k]) >> 32 == names[e["event_slot_45_name"]]
    g.close()


def test_serf_reap_handler(kats):
    """The Reaper (reap.rs:41-131; Reaper::run, base.rs:580-601) at now = 100 s with
    tombstone_timeout 6 s and recent_intent_timeout 7 s: of three left members aged 0, 5 and
    10 s two remain; of the intents alice (join, 0 s), bob (join, 10 s), carol (leave, 0 s),
    doug (leave, 10 s) alice and carol are kept.  The engine's clock is the round number, so
    the left members are made by memberlist NotifyLeave of Leaving members in rounds 90, 95
    and 100 (Leaving -> Left stamps leave_time), the intents by notify_message at set_now times."""
    k = kats["merge"]["serf_reap_handler"]
    ages, intents = k["left_ages_s"], k["intents"]
    s = len(ages) + len(intents)
    g = engine(n=s + 4, s=s)
    now = 100
    for i in range(len(ages)):
        g.set_view(0, i, G.KIND_KNOWN, G.STATUS_LEAVING, 3)
    for i, age in sorted(enumerate(ages), key=lambda x: -x[1]):
        g.round(now - age, ml(i, G.ML_LEAVE))
    for j, (_node, ty, lt, age) in enumerate(intents):
        g.set_now(now - age)
        g.apply_batch(msgs([(0, G.MSG_JOIN if ty == "join" else G.MSG_LEAVE, len(ages) + j, lt, 0, 0)]))
    for i, age in enumerate(ages):
        kd, st, lt, tm = entry(g, 0, i)
        assert (kd, st, tm) == (G.KIND_KNOWN, G.STATUS_LEFT, now - age)
    d0 = int(g.members()["digest"][0])
    g.reap(now, 1 << 30, k["tombstone_timeout_s"], k["recent_intent_timeout_s"])
    left = [entry(g, 0, i)[:2] == (G.KIND_KNOWN, G.STATUS_LEFT) for i in range(len(ages))]
    assert sum(left) == k["expect_left_remaining"]
    kept = [node for j, (node, *_r) in enumerate(intents) if entry(g, 0, len(ages) + j)[0] != G.KIND_UNKNOWN]
    assert kept == k["expect_intents_kept"]
    assert int(g.members()["digest"][0]) != d0  # the Reap member event
    g.close()


# ------------------------------------------------------------------ dissemination (event.rs)
def test_user_event_old_message(kats):
    """After witnessing 1512 the event clock is past the buffer: an event at ltime 1 is
    too old (event.rs:6-29)."""
    k = kats["dissemination"]["user_event_old_message"]
    g = engine()
    g.set_clocks(0, 1, k["witness"] + 1, 1)  # event_clock.witness(1512)
    flags, _ = g.apply_batch(msgs([(0, G.MSG_USER_EVENT, 0, k["ltime"], 7, 0)]))
    assert bool(flags[0] & G.F_REBROADCAST) == k["expect"] and not flags[0] & G.F_DELIVER
    g.close()


def test_user_event_same_clock(kats):
    """Three events at one ltime with distinct (name, payload) are all delivered and
    rebroadcast, in arrival order; a repeat is not (event.rs:32-74)."""
    k = kats["dissemination"]["user_event_same_clock"]
    g = engine()
    g.set_delivery_log(16)
    names, payloads, keys = {}, {}, []
    for _lt, name, payload in k["events"]:
        keys.append((names.setdefault(name, len(names) + 1) << 32) | payloads.setdefault(payload, len(payloads) + 1))
    flags, _ = g.apply_batch(msgs([(0, G.MSG_USER_EVENT, 0, lt, key, 0) for (lt, _n, _p), key in zip(k["events"], keys)]))
    assert [bool(f & G.F_REBROADCAST) for f in flags] == k["expect"]
    d = g.deliveries()
    inv_n = {v: kk for kk, v in names.items()}
    inv_p = {v: kk for kk, v in payloads.items()}
    assert [[inv_n[int(x) >> 32], inv_p[int(x) & 0xFFFFFFFF]] for x in d["key"]] == k["delivered"]
    assert np.all(d["kind"] == G.DELIVERY_USER_EVENT) and np.all(d["ltime"] == 1)
    flags, _ = g.apply_batch(msgs([(0, G.MSG_USER_EVENT, 0, 1, keys[1], 0)]))
    assert flags[0] == 0
    g.close()


def test_query_old_message(kats):
    """After witnessing 1512 the query clock is past the buffer: a query at ltime 1 is
    dropped, and -- the reference's comparison of the buffer length (base.rs:999) -- so is a
    current one (event.rs:653-687)."""
    k = kats["dissemination"]["query_old_message"]
    g = engine()
    g.set_clocks(0, 1, 1, k["witness"] + 1)
    flags, _ = g.apply_batch(msgs([(0, G.MSG_QUERY, 0, k["ltime"], k["id"], 0),
                                   (0, G.MSG_QUERY, 0, k["witness"] + 1, 99, 0)]))
    assert bool(flags[0] & G.F_REBROADCAST) == k["expect"] and flags[1] == 0
    g.close()


def test_query_same_clock(kats):
    """Queries at one ltime with distinct ids are rebroadcast once each; the slot keeps
    the ids in arrival order (event.rs:690-775)."""
    k = kats["dissemination"]["query_same_clock"]
    g = engine()
    flags, _ = g.apply_batch(msgs([(0, G.MSG_QUERY, 0, lt, qid, 0) for lt, qid, _name in k["queries"]]))
    assert [bool(f & G.F_REBROADCAST) for f in flags] == k["expect"]
    *_e, qbl, qbc, qbi = g.buffers()
    slot_k = g.cfg.slot_k
    ids = [int(x) for x in qbi[slot_k:slot_k + int(qbc[1])]]
    delivered = {qid: name for _lt, qid, name in k["queries"]}
    assert [delivered[i] for i in ids] == k["delivered"]
    g.close()


def test_delivery_log_full_width_ltime():
    """A user event's Lamport time comes off the wire as a full u64: one at or above 2^62 is
    logged as a user event with its time intact (the log's kind and cc flags live in a byte
    of their own), next to a member event of the same member."""
    g = engine()
    g.set_delivery_log(8)
    big = (1 << 62) + 5
    g.set_view(0, 1, G.KIND_KNOWN, G.STATUS_FAILED, 3)
    flags, _ = g.apply_batch(msgs([(0, G.MSG_USER_EVENT, 0, big, 7 << 32, 1),
                                   (0, G.MSG_LEAVE, 1, 9, 0, 0)]))  # Failed -> Left: a Leave member event
    assert flags[0] & G.F_DELIVER and flags[1] & G.F_MEMBER_EVENT
    d = g.deliveries()
    assert len(d) == 2
    assert (int(d[0]["ltime"]), int(d[0]["key"]), int(d[0]["cc"]), int(d[0]["kind"])) == \
        (big, 7 << 32, 1, G.DELIVERY_USER_EVENT)
    assert (int(d[1]["ltime"]), int(d[1]["key"]), int(d[1]["kind"])) == (1, 1, G.DELIVERY_MEMBER_EVENT)
    g.close()


# ------------------------------------------------------------------ origination size limits
def _originate(g, act, name_len, payload_len, key=7):
    a = np.zeros(1, G.ACTION_DTYPE)
    a["member"], a["act"], a["name_len"], a["payload_len"], a["key"] = 0, act, name_len, payload_len, key
    return a


def _sized(k, name):
    return k[k[name]["payload_len"]]["value"]


def _nothing_moved(g, before):
    """no clock moved, nothing delivered, queued or sent anywhere"""
    after = g.members()
    for f in ("clock", "event_clock", "query_clock", "digest"):
        assert np.array_equal(after[f], before[f]), f
    assert len(g.deliveries()) == 0
    rumor, *_x, next_seq = g.queues()
    assert np.all(rumor == 0xFFFFFFFF) and np.all(next_seq == 0)


@pytest.mark.parametrize("payload,expect", [("limit", G.ERR_USER_EVENT_LIMIT), (486, G.ERR_RAW_USER_EVENT_TOO_LARGE),
                                            (487, G.ERR_USER_EVENT_LIMIT)])
def test_serf_event_user_size_limit(kats, payload, expect):
    """Serf::user_event with "this is too large an event" and a payload of
    max_user_event_size bytes fails with UserEventLimitTooLarge before the event clock
    moves (event.rs:506-525; api.rs:255-262): status, event clock, deliveries, queues and
    every member's digest unchanged.  The boundary: name + payload == the limit (26 + 486)
    passes the first check and fails the encoded-length one (RawUserEventTooLarge,
    api.rs:281-283); one byte more fails the first."""
    d = kats["dissemination"]
    k = d["serf_event_user_size_limit"]
    limit = _sized(d, "serf_event_user_size_limit")
    g = engine(max_user_event_size=limit)
    g.set_delivery_log(8)
    before = g.members()
    g.round(0, None, _originate(g, G.ACT_USER_EVENT, len(k["name"]), limit if payload == "limit" else payload))
    st = int(g.action_status()[0])
    assert st == expect
    assert k["expect_error_contains"] in G.serf_error_text(st, g.cfg, size=0)
    _nothing_moved(g, before)
    g.close()


def test_user_event_within_limit_originates(kats):
    """A small event passes every check: the event clock moves, the origin delivers it and
    queues it (the control for the size-limit cases)."""
    g = engine()
    g.set_delivery_log(8)
    g.round(0, None, _originate(g, G.ACT_USER_EVENT, 8, 32))
    assert g.action_status()[0] == G.ACT_OK
    assert int(g.members()["event_clock"][0]) == 2 and len(g.deliveries()) >= 1
    g.close()


@pytest.mark.parametrize("case", ["serf_query_size_limit", "serf_query_size_limit_increased"])
def test_serf_query_size_limit(kats, case):
    """query_in with "this is too large a query" and a payload of query_size_limit bytes:
    QueryTooLarge at the default limit (event.rs:1070-1085), accepted at twice the limit
    (event.rs:1087-1100; base.rs:916-921).  A rejected query queues nothing and moves no
    clock; an accepted one is handled locally and queued."""
    d = kats["dissemination"]
    k = d[case]
    limit = _sized(d, case)
    g = engine(query_size_limit=limit * k["query_size_limit_factor"])
    before = g.members()
    g.round(0, None, _originate(g, G.ACT_QUERY, len(k["name"]), limit))
    st = int(g.action_status()[0])
    if k.get("expect_ok"):
        assert st == G.ACT_OK
        *_x, next_seq = g.queues()
        assert int(next_seq.reshape(-1, 3)[0, 1]) == 1  # the query entered the origin's query queue
    else:
        assert st == G.ERR_QUERY_TOO_LARGE
        assert k["expect_error_contains"] in G.serf_error_text(st, g.cfg, size=0)
        _nothing_moved(g, before)
    g.close()


def test_user_event_size_limit_at_create():
    """max_user_event_size above USER_EVENT_SIZE_LIMIT fails at create (base.rs:69-70)."""
    with pytest.raises(G._lib.EngineError) as e:
        engine(max_user_event_size=G.USER_EVENT_SIZE_LIMIT + 1)
    assert e.value.code == G.ERR_USER_EVENT_LIMIT
