"""memberlist SWIM model: the oracle's restatement of aliveNode /
suspectNode / deadNode / refute / suspicion timers on hand-worked cases, and the host
side of the C ABI (no GPU).  memberlist-core 0.2 is not vendored in the reference, so
these cases follow memberlist's published state machine: PARITY UNPINNED."""
import ctypes as C
import math

import numpy as np
import pytest

import oracle_ffi as O
from ruserf_amd import swim as W

A, SU, D, LF, UN = W.ALIVE, W.SUSPECT, W.DEAD, W.LEFT, W.UNKNOWN
RB, RF, NJ, NL, SS, CF = (W.F_REBROADCAST, W.F_REFUTE, W.F_NOTIFY_JOIN, W.F_NOTIFY_LEAVE, W.F_SUSPECT,
                          W.F_CONFIRM)


def msg(rcv, subj, inc, typ, frm=99):
    m = np.zeros(1, dtype=W.MSG_DTYPE)
    m["receiver"], m["subject"], m["incarnation"], m["type"], m["from"] = rcv, subj, inc, typ, frm
    return m


def world(state0, inc0, k=2, timeouts=(100, 80, 60, 60, 60), self_inc=1):
    # members 0..3 receive; subject s is member 10 + s, except subject 3 = member 0 (self of receiver 0)
    S = len(state0)
    subj = np.array([10 + s for s in range(S)], np.uint32)
    subj[3] = 0
    return O.OracleSwim(0, 4, S, k, timeouts, subj, state0, inc0, self_inc), subj


def test_alive_unknown_node_is_added_dead_then_incarnation_checked():
    w, _ = world([UN, A, A, A], [0, 1, 1, 1])
    f, _ = w.apply(msg(1, 0, 0, W.MSG_ALIVE), now=5)  # incarnation 0 <= 0: added as dead, bail
    d = w.dump()
    assert f[0] == 0 and d["state"][1, 0] == D and d["incarnation"][1, 0] == 0
    f, _ = w.apply(msg(1, 0, 3, W.MSG_ALIVE), now=6)
    d = w.dump()
    assert f[0] == RB | NJ and d["state"][1, 0] == A and d["incarnation"][1, 0] == 3 and d["change"][1, 0] == 6
    f, _ = w.apply(msg(1, 0, 3, W.MSG_ALIVE), now=7)  # same incarnation: old news
    assert f[0] == 0
    w.close()


def test_suspect_confirmations_and_timeout():
    w, _ = world([A, A, A, A], [2, 2, 2, 2], k=2, timeouts=(100, 80, 60, 60, 60))
    f, _ = w.apply(msg(2, 1, 1, W.MSG_SUSPECT, frm=7), now=10)  # older incarnation
    assert f[0] == 0
    f, _ = w.apply(msg(2, 1, 2, W.MSG_SUSPECT, frm=7), now=10)
    assert f[0] == RB | SS
    assert w.dump()["state"][2, 1] == SU
    assert w.apply(msg(2, 1, 2, W.MSG_SUSPECT, frm=7), now=11)[0][0] == 0  # the first accuser again
    assert w.apply(msg(2, 1, 2, W.MSG_SUSPECT, frm=8), now=12)[0][0] == RB | CF
    assert w.apply(msg(2, 1, 5, W.MSG_SUSPECT, frm=9), now=13)[0][0] == RB | CF
    assert w.apply(msg(2, 1, 5, W.MSG_SUSPECT, frm=6), now=14)[0][0] == 0  # k = 2 confirmations reached
    d = w.dump()
    assert d["n_confirm"][2, 1] == 2 and d["incarnation"][2, 1] == 2  # a confirmation does not move inc
    assert w.tick(10 + 59) == 0
    assert w.tick(10 + 60) == 1  # timeout[2] = 60 after two confirmations
    d = w.dump()
    assert d["state"][2, 1] == D and d["change"][2, 1] == 70 and d["n_confirm"][2, 1] == 0
    w.close()


def test_alive_with_newer_incarnation_clears_suspicion():
    w, _ = world([A, A, A, A], [2, 2, 2, 2])
    w.apply(msg(1, 2, 2, W.MSG_SUSPECT), now=1)
    assert w.apply(msg(1, 2, 2, W.MSG_ALIVE), now=2)[0][0] == 0  # not newer: the suspicion stays
    assert w.dump()["state"][1, 2] == SU
    assert w.apply(msg(1, 2, 3, W.MSG_ALIVE), now=3)[0][0] == RB  # suspect -> alive: no join notification
    d = w.dump()
    assert d["state"][1, 2] == A and d["incarnation"][1, 2] == 3 and d["change"][1, 2] == 3
    assert w.tick(10_000) == 0
    w.close()


def test_refutations_about_self():
    # receiver 0 is subject 3; m.incarnation = 1, its own entry incarnation 1
    w, _ = world([A, A, A, A], [1, 1, 1, 1], self_inc=1)
    f, r = w.apply(msg(0, 3, 5, W.MSG_SUSPECT), now=1)
    assert f[0] == RF and r[0] == 6  # accused 5 >= 2: skip to 6
    d = w.dump()
    assert d["state"][0, 3] == A and d["incarnation"][0, 3] == 6 and d["self_incarnation"][0] == 6
    f, r = w.apply(msg(0, 3, 2, W.MSG_DEAD), now=2)  # older than 6: ignored
    assert f[0] == 0
    f, r = w.apply(msg(0, 3, 6, W.MSG_DEAD), now=3)
    assert f[0] == RF and r[0] == 7  # nextIncarnation 7 > accused 6
    f, r = w.apply(msg(0, 3, 7, W.MSG_ALIVE), now=4)  # an equal alive about ourselves: nothing
    assert f[0] == 0
    f, r = w.apply(msg(0, 3, 9, W.MSG_ALIVE), now=5)  # a newer one: refute past it
    assert f[0] == RF and r[0] == 10
    w.set_left(0)
    f, r = w.apply(msg(0, 3, 10, W.MSG_DEAD, frm=0), now=6)  # we left: not refuted, marked left
    assert f[0] == RB | NL and w.dump()["state"][0, 3] == LF
    w.close()


def test_dead_and_left():
    w, subj = world([A, SU, D, A], [1, 1, 1, 1])
    f, _ = w.apply(msg(1, 0, 1, W.MSG_DEAD, frm=int(subj[0])), now=4)  # from the node itself: left
    assert f[0] == RB | NL and w.dump()["state"][1, 0] == LF
    f, _ = w.apply(msg(1, 1, 1, W.MSG_DEAD, frm=5), now=4)  # suspect -> dead
    assert f[0] == RB | NL and w.dump()["state"][1, 1] == D
    assert w.apply(msg(1, 2, 4, W.MSG_DEAD, frm=5), now=4)[0][0] == 0  # already dead
    assert w.apply(msg(1, 2, 4, W.MSG_SUSPECT, frm=5), now=4)[0][0] == 0  # suspect of a dead node
    f, _ = w.apply(msg(1, 2, 2, W.MSG_ALIVE), now=8)  # dead -> alive: join notification
    assert f[0] == RB | NJ
    w.close()


def test_suspicion_timeouts_formula():
    t = W.suspicion_timeouts(2, 5000, 30000)
    # memberlist remainingSuspicionTime: max - log(c+1)/log(k+1) * (max - min), floored
    assert t[0] == 30000
    assert t[1] == math.floor(30000 - math.log(2) / math.log(3) * 25000)
    assert t[2] == 5000 and t[3] == 5000
    assert W.suspicion_timeouts(0, 5000, 30000) == [5000] * 5


def test_create_rejects_bad_config_without_gpu():
    from ruserf_amd._lib import lib
    W._declare(lib())
    h = C.c_void_p()
    bad = W.RsfSwimCfg(n_members=10, shard_lo=4, shard_hi=2, n_subjects=3, suspicion_k=2)
    assert lib().rsf_swim_create(C.byref(h), C.byref(bad), 0) != 0
    bad = W.RsfSwimCfg(n_members=10, shard_lo=0, shard_hi=10, n_subjects=3, suspicion_k=9)
    assert lib().rsf_swim_create(C.byref(h), C.byref(bad), 0) != 0


@pytest.mark.parametrize("seed", [1, 2])
def test_oracle_batch_is_order_of_messages(seed):
    """Receivers are independent: applying a batch in one call or split per receiver gives
    the same state (what the GPU's receiver-parallel apply relies on)."""
    import swim_cases as SC
    subj, st0, inc0 = SC.random_world(64, 12, seed)
    t = W.suspicion_timeouts(2, 50, 300)
    a = O.OracleSwim(0, 16, 12, 2, t, subj, st0, inc0)
    b = O.OracleSwim(0, 16, 12, 2, t, subj, st0, inc0)
    rng = np.random.default_rng(seed)
    m = SC.random_batch(rng, 0, 16, 12, subj, 400)
    fa, _ = a.apply(m, 100)
    fb = np.zeros(len(m), np.int32)
    for r in range(16):
        idx = np.nonzero(m["receiver"] == r)[0]
        if len(idx):
            fb[idx] = b.apply(m[idx], 100)[0]
    assert np.array_equal(fa, fb)
    for k, v in a.dump().items():
        assert np.array_equal(v, b.dump()[k]), k
    a.close()
    b.close()
