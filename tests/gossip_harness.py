"""Builds matching (GPU engine, CPU oracle world) pairs and compares their full
state bit for bit.  Test infrastructure: the oracle is only the checker."""
import ctypes as C

import numpy as np

import oracle_ffi as O

L = O.lib()


def queue_depths(cfg):
    """each queue's capacity: queue_cap, or the deeper queue_depth (head + HBM tail)"""
    d = getattr(cfg, "queue_depth", None) or (0, 0, 0)
    return [int(x) if x else cfg.queue_cap for x in d]


def oracle_world(cfg, subj_member, views):
    qd = queue_depths(cfg)
    wc = O.WorldCfg(n=cfg.n_members, s=cfg.n_subjects, qcap=max(qd), ebuf=cfg.event_buffer_size,
                    qbuf=cfg.query_buffer_size, slot_k=cfg.slot_k, fanout=cfg.fanout, limit=cfg.gossip_limit,
                    overhead=cfg.gossip_overhead, retransmit_mult=cfg.retransmit_mult, max_refute=cfg.max_refute,
                    cap_rumors=cfg.max_rumors, seed=cfg.seed,
                    max_user_event_size=getattr(cfg, "max_user_event_size", 512),
                    query_size_limit=getattr(cfg, "query_size_limit", 1024))
    wc.qdepth[:] = qd
    w = O.World()
    assert L.orc_world_init(C.byref(w), C.byref(wc)) == 0
    n, s = cfg.n_members, cfg.n_subjects
    sm = O.arr(w.subj_member, s, np.uint32)
    sm[:] = subj_member
    ms = O.arr(w.member_subj, n, np.int32)
    ms[subj_member] = np.arange(s, dtype=np.int32)
    kind, status, ltime = views
    O.arr(w.v_kind, n * s, np.uint8).reshape(n, s)[:] = kind[None, :]
    O.arr(w.v_status, n * s, np.uint8).reshape(n, s)[:] = status[None, :]
    O.arr(w.v_ltime, n * s, np.uint64).reshape(n, s)[:] = ltime[None, :]
    return w


def oracle_round(w, t, ml, acts, threads=1):
    ml = np.ascontiguousarray(ml, dtype=np.dtype([("subject", "<u4"), ("kind", "<u4"), ("set_alive", "<u4"),
                                                  ("_r", "<u4")]))
    acts = np.ascontiguousarray(acts)
    rc = L.orc_world_round_mt(C.byref(w), t, ml.ctypes.data_as(C.POINTER(O.MlEvent)), len(ml),
                              acts.ctypes.data_as(C.POINTER(O.Action)), len(acts), threads)
    assert rc == 0


def world_width(w):
    """slots [0, hwm) of every oracle queue hold all its live items"""
    return max(1, int(O.arr(w.q_hwm, w.n * 3, np.uint32).max()))


def world_state(w, lo=0, hi=None, width=None):
    n, s, q = w.n, w.s, w.qcap
    hi = n if hi is None else hi
    sl = slice(lo, hi)
    if width is not None:  # deep queues: only the slots that can hold items (width >= the hwm)
        assert width >= world_width(w)
        qs = lambda p, t: np.ascontiguousarray(O.arr(p, n * 3 * q, t).reshape(n, 3, q)[sl, :, :width]).reshape(hi - lo, -1)  # noqa: E731
    else:
        qs = lambda p, t: O.arr(p, n * 3 * q, t).reshape(n, 3 * q)[sl]  # noqa: E731
    st = {
        "clock": O.arr(w.clock, n, np.uint64)[sl],
        "event_clock": O.arr(w.eclock, n, np.uint64)[sl],
        "query_clock": O.arr(w.qclock, n, np.uint64)[sl],
        "digest": O.arr(w.digest, n, np.uint64)[sl],
        "err": O.arr(w.err, n, np.uint32)[sl],
        "serf_state": O.arr(w.serf_state, n, np.uint8)[sl],
        "v_ltime": O.arr(w.v_ltime, n * s, np.uint64).reshape(n, s)[sl],
        "v_status": O.arr(w.v_status, n * s, np.uint8).reshape(n, s)[sl],
        "v_kind": O.arr(w.v_kind, n * s, np.uint8).reshape(n, s)[sl],
        "v_time": O.arr(w.v_time, n * s, np.uint32).reshape(n, s)[sl],
        "q_rumor": qs(w.q_rumor, np.uint32),
        "q_seq": qs(w.q_seq, np.uint32),
        "q_tx": qs(w.q_tx, np.uint16),
        "q_len": qs(w.q_len, np.uint16),
        "q_next_seq": O.arr(w.q_next_seq, n * 3, np.uint32).reshape(n, 3)[sl],
        "eb_ltime": O.arr(w.eb_ltime, n * w.ebuf, np.uint64).reshape(n, -1)[sl],
        "eb_cnt": O.arr(w.eb_cnt, n * w.ebuf, np.uint32).reshape(n, -1)[sl],
        "eb_keys": O.arr(w.eb_keys, n * w.ebuf * w.slot_k, np.uint64).reshape(n, -1)[sl],
        "qb_ltime": O.arr(w.qb_ltime, n * w.qbuf, np.uint64).reshape(n, -1)[sl],
        "qb_cnt": O.arr(w.qb_cnt, n * w.qbuf, np.uint32).reshape(n, -1)[sl],
        "qb_ids": O.arr(w.qb_ids, n * w.qbuf * w.slot_k, np.uint32).reshape(n, -1)[sl],
        "q_pruned": O.arr(w.q_pruned, n, np.uint32)[sl],
        "q_expired": O.arr(w.q_expired, n, np.uint32)[sl],
    }
    return st


def engine_state(g, width=None):
    n, s, q = g.n_loc, g.cfg.n_subjects, g.cfg.queue_cap
    m = g.members()
    lt, stt, kd, vt = g.view(with_time=True)
    r, sq, tx, ln, ns = g.queues(width)
    if width is not None:
        assert g.max_live <= width, (g.max_live, width)
    ebl, ebc, ebk, qbl, qbc, qbi = g.buffers()
    return {
        "clock": m["clock"], "event_clock": m["event_clock"], "query_clock": m["query_clock"],
        "digest": m["digest"], "err": m["err"], "serf_state": m["serf_state"],
        "v_ltime": lt.reshape(n, s), "v_status": stt.reshape(n, s), "v_kind": kd.reshape(n, s),
        "v_time": vt.reshape(n, s),
        "q_rumor": r.reshape(n, -1), "q_seq": sq.reshape(n, -1), "q_tx": tx.reshape(n, -1),
        "q_len": ln.reshape(n, -1), "q_next_seq": ns.reshape(n, 3),
        "eb_ltime": ebl.reshape(n, -1), "eb_cnt": ebc.reshape(n, -1), "eb_keys": ebk.reshape(n, -1),
        "qb_ltime": qbl.reshape(n, -1), "qb_cnt": qbc.reshape(n, -1), "qb_ids": qbi.reshape(n, -1),
        "q_pruned": g.pruned(),
        "q_expired": g.expired(),
    }


def normalize_queues(st, qcap=None):
    """Queue slot ORDER is an implementation detail (the oracle fills the first free
    slot, the kernels keep each queue sorted in send order); the queue CONTENT is
    what the reference defines.  Canonical form: each queue's live items sorted by
    (transmits, len desc, seq desc), free slots after them and zeroed."""
    st = dict(st)
    r = st["q_rumor"]
    n, w = r.shape
    q = qcap or (w // 3)
    rr = r.reshape(n, 3, q)
    sq = st["q_seq"].reshape(n, 3, q).astype(np.uint64)
    tx = st["q_tx"].reshape(n, 3, q).astype(np.uint64)
    ln = st["q_len"].reshape(n, 3, q).astype(np.uint64)
    empty = rr == 0xFFFFFFFF
    key = (tx << 48) | ((0xFFFF - ln) << 32) | (0xFFFFFFFF - sq)
    key = np.where(empty, np.uint64(0xFFFFFFFFFFFFFFFF), key)
    order = np.argsort(key, axis=2, kind="stable")
    for k in ["q_rumor", "q_seq", "q_tx", "q_len"]:
        a = st[k].reshape(n, 3, q)
        a = np.take_along_axis(a, order, axis=2).copy()
        if k != "q_rumor":
            a[np.take_along_axis(empty, order, axis=2)] = 0
        st[k] = a.reshape(n, w)
    return st


def deep_states(g, w):
    """(engine, oracle) states of a deep-queue pair with only the queue slots in use compared"""
    width = world_width(w)
    return engine_state(g, width), world_state(w, width=width)


def assert_same(a, b, ctx=""):
    a = normalize_queues(a)
    b = normalize_queues(b)
    for k in a:
        x, y = np.asarray(a[k]), np.asarray(b[k])
        if not np.array_equal(x, y):
            bad = np.argwhere(x != y)
            raise AssertionError(f"{ctx}: field {k} differs at {len(bad)} places, first {bad[:5].tolist()}: "
                                 f"got {x[tuple(bad[0])]} expected {y[tuple(bad[0])]}")


def oracle_rumors(w):
    """the rumor ring's slots up to the cursor"""
    return [(w.rumors[i].type, w.rumors[i].ltime, w.rumors[i].subject, w.rumors[i].key, w.rumors[i].msg_len)
            for i in range(w.n_rumors)]


def oracle_push_pull(w, pairs, is_join=False, event_join_ignore=False):
    pairs = np.ascontiguousarray(pairs)
    recv = np.ascontiguousarray(pairs["receiver"], dtype=np.uint32)
    send = np.ascontiguousarray(pairs["sender"], dtype=np.uint32)
    assert L.orc_push_pull(C.byref(w), O.ptr(recv, C.c_uint32), O.ptr(send, C.c_uint32), len(pairs),
                           int(is_join), int(event_join_ignore)) == 0


def matching_pairs(rng, members, both=True):
    """A random perfect matching over `members` as push/pull (receiver, sender) rows:
    each exchange a<->b contributes (a<-b) and (b<-a)."""
    from ruserf_amd.gossip import PP_PAIR_DTYPE
    m = rng.permutation(np.asarray(members, dtype=np.uint32))
    m = m[: len(m) // 2 * 2].reshape(-1, 2)
    rows = [(a, b) for a, b in m] + ([(b, a) for a, b in m] if both else [])
    out = np.zeros(len(rows), PP_PAIR_DTYPE)
    if rows:
        out["receiver"] = [r[0] for r in rows]
        out["sender"] = [r[1] for r in rows]
    return out
