"""GPU parity of the snapshot log, the restart from a snapshot and the Reconnector
against the CPU oracle (tests/test_snapshot.py pins the oracle to the reference's
snapshotter tests).  Bit-exact: the snapshotters' alive sets and clocks, every member's
encoded snapshot file, the member state after restarts, the Reconnector's targets and
the state after its joins."""
import ctypes as C

import numpy as np
import pytest

import gossip_harness as H
import oracle_ffi as O
from ruserf_amd import gossip as G
from ruserf_amd import workload as W

pytestmark = pytest.mark.gpu
L = O.lib()


def _setup(n, rounds, seed, false_failures=0):
    subj, acts, ml = W.churn_workload(n, rounds, events_per_round=20, queries_per_round=4, seed=seed)
    s = len(subj)
    rng_u = np.random.default_rng(seed + 1)
    for t in range(rounds):  # NotifyUpdate -> handle_node_update (Update member events)
        extra = np.zeros(3, dtype=ml[t].dtype)
        extra["subject"] = rng_u.choice(s, 3, replace=False)
        extra["kind"] = G.ML_UPDATE
        extra["set_alive"] = 2
        ml[t] = np.concatenate([ml[t], extra])
    if false_failures:
        # memberlist marks some up members failed (set_alive 2: liveness unchanged), so a
        # Reconnector try can succeed
        rng = np.random.default_rng(seed)
        for t in range(1, rounds, 3):
            extra = np.zeros(false_failures, dtype=ml[t].dtype)
            extra["subject"] = rng.choice(s, false_failures, replace=False)
            extra["kind"] = G.ML_LEAVE
            extra["set_alive"] = 2
            ml[t] = np.concatenate([ml[t], extra])
    cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=24, gossip_limit=400, max_rumors=1 << 15,
                         event_buffer_size=64, query_buffer_size=64, slot_k=8, seed=seed)
    views = W.initial_views(s)
    g = G.GossipEngine(cfg)
    g.set_subjects(subj)
    g.init_views(*views)
    w = H.oracle_world(cfg, subj, views)
    return g, w, cfg, subj, acts, ml


def oracle_files(w, members):
    out = []
    for m in members:
        size = L.orc_world_snapshot_encode(C.byref(w), int(m), None)
        buf = np.zeros(max(1, size), np.uint8)
        L.orc_world_snapshot_encode(C.byref(w), int(m), O.ptr(buf, C.c_uint8))
        out.append(bytes(buf[:size]))
    return out


def check_snapshots(g, w, ctx):
    bits, sn = g.snapshot_state()
    n = w.n
    ob = O.arr(w.snap_bits, n * w.snap_w, np.uint32).reshape(n, w.snap_w)
    osn = O.arr(w.snap_sn, n * 4, np.uint64).reshape(n, 4)
    assert np.array_equal(bits, ob), ctx
    assert np.array_equal(sn, osn), ctx
    offs, blob = g.snapshot_files()
    want = oracle_files(w, range(n))
    assert int(offs[-1]) == sum(len(f) for f in want), ctx
    for m in range(n):
        assert bytes(blob[offs[m]:offs[m + 1]]) == want[m], f"{ctx}: member {m}"


@pytest.mark.parametrize("rejoin", [False, True])
def test_snapshot_rounds_and_restart_bit_exact(rejoin):
    n, rounds = 2500, 16
    g, w, cfg, subj, acts, ml = _setup(n, rounds, seed=31)
    g.enable_snapshot(rejoin)
    assert L.orc_world_enable_snapshot(C.byref(w), int(rejoin)) == 0
    check_snapshots(g, w, "enabled")
    rng = np.random.default_rng(5)
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t])
        if t in (5, 11):
            check_snapshots(g, w, f"round {t}")
            # restart a batch from their own files (one from a damaged file: unchanged)
            members = np.sort(rng.choice(n, 40, replace=False)).astype(np.uint32)
            files = oracle_files(w, members)
            files[3] = files[3][:-4]
            res = g.restart(members, files)
            for i, m in enumerate(members):
                a = np.frombuffer(files[i] or b"\0", np.uint8).copy()
                want = L.orc_world_restart(C.byref(w), int(m), O.ptr(a, C.c_uint8), len(files[i]))
                assert res[i] == want, (t, int(m))
            assert res[3] < 0 and np.count_nonzero(res == 1) > 0
        H.assert_same(H.engine_state(g), H.world_state(w), f"round {t}")
    check_snapshots(g, w, "end")
    _, sn = g.snapshot_state()
    assert np.count_nonzero(sn[:, 3] & 1) > 0  # some members left (recording stopped)
    g.close()
    L.orc_world_free(C.byref(w))


def test_reconnect_bit_exact():
    n, rounds = 3000, 15
    g, w, cfg, subj, acts, ml = _setup(n, rounds, seed=47, false_failures=6)
    g.enable_snapshot(False)
    assert L.orc_world_enable_snapshot(C.byref(w), 0) == 0
    tried = joined = 0
    for t in range(rounds):
        g.round(t, ml[t], acts[t])
        H.oracle_round(w, t, ml[t], acts[t])
        if t % 2 == 1:
            tgt = g.reconnect_targets(t)
            want = np.zeros(n, np.uint32)
            joined += L.orc_world_reconnect(C.byref(w), t, O.ptr(want, C.c_uint32))
            assert np.array_equal(tgt, want), f"tick {t}"
            tried += int(np.count_nonzero(want != 0xFFFFFFFF))
        H.assert_same(H.engine_state(g), H.world_state(w), f"round {t}")
    check_snapshots(g, w, "end")
    assert tried > 0 and joined > 0
    g.close()
    L.orc_world_free(C.byref(w))
