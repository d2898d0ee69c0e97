"""memberlist's probe loop feeding the coordinate clients and the failure detector
(ruserf_amd.probe.ProbeLoop).  memberlist is not vendored by the
reference: the probe schedule and the suspicion rules are PARITY UNPINNED; what is
checked bit for bit:
  * the wire path (ack payload bytes -> notify_ping_complete) equals the table path;
  * every acked probe is CoordinateClient::update against the oracle's clients, with
    the target's previous-round coordinate; a timed-out probe leaves the member as is;
  * timed-out probes of tracked subjects suspect them exactly as the oracle's
    suspectNode from the prober, and the suspicion timers fire identically.
"""
import ctypes as C

import numpy as np
import pytest
import torch

import oracle_ffi as O
from ruserf_amd import CoordinateClients, CoordinateOptions
from ruserf_amd import swim as SW
from ruserf_amd.probe import ProbeLoop

pytestmark = pytest.mark.gpu
L = O.lib()
SEED = 0x5EED5EED


def _table(g):
    from ruserf_amd.dist import hbm_tensor
    ptr, stride = g.table_ptr()
    return hbm_tensor(ptr, g.n * stride, "<f8").view(g.n, stride)


def _up(n, frac_down, seed):
    rng = np.random.default_rng(seed)
    up = np.ones(n, np.uint8)
    up[rng.choice(n, int(n * frac_down), replace=False)] = 0
    return up


def test_wire_path_equals_table_path():
    n, peers, rounds = 20_000, 16, 10
    up = torch.from_numpy(_up(n, 0.1, 1)).cuda()
    a = CoordinateClients(n, peers, CoordinateOptions(), seed=SEED)
    b = CoordinateClients(n, peers, CoordinateOptions(), seed=SEED)
    pa, pb = ProbeLoop(a, wire=True), ProbeLoop(b, wire=False)
    for r in range(rounds):
        pa.round(r, up)
        pb.round(r, up)
        torch.cuda.synchronize()
        acked = pa.acked.cpu().numpy().astype(bool)
        assert np.array_equal(acked, pb.acked.cpu().numpy().astype(bool))
        sa, sb = pa.status.cpu().numpy(), pb.status.cpu().numpy()
        assert np.all(sa[acked] == sb[acked])
        assert np.all(sa[~acked] == 4)  # RSF_SKIPPED: no ack, no update
        assert np.all(sb[~acked] != 0)  # rtt > 10 s: rejected, member unchanged
        assert torch.equal(_table(a)[:, :11].view(torch.int64), _table(b)[:, :11].view(torch.int64)), r
    a.close()
    b.close()


def test_probe_loop_matches_oracle_clients():
    n, peers, rounds = 3000, 16, 8
    up_np = _up(n, 0.15, 2)
    up = torch.from_numpy(up_np).cuda()
    oo = O.default_opts()
    clients = []
    for _ in range(n):
        c = O.Client()
        assert L.orc_client_init(C.byref(c), C.byref(oo), peers) == 0
        clients.append(c)
    g = CoordinateClients(n, peers, CoordinateOptions(), seed=SEED)
    loop = ProbeLoop(g, wire=True)
    gp = torch.empty(n, dtype=torch.int32, device="cuda")
    gr = torch.empty(n, dtype=torch.int64, device="cuda")
    for r in range(rounds):
        prev = _table(g).clone().cpu().numpy()
        g.gen_probes(r, gp.data_ptr(), gr.data_ptr())
        loop.round(r, up)
        torch.cuda.synchronize()
        peer = loop.peer.cpu().numpy().astype(np.int64)
        acked = loop.acked.cpu().numpy().astype(bool)
        rtt = loop.rtt.cpu().numpy().view(np.uint64)
        assert np.array_equal(peer, gp.cpu().numpy().astype(np.int64))
        want_ack = (up_np.astype(bool) & up_np[peer].astype(bool)) & (peer != np.arange(n))
        assert np.array_equal(acked, want_ack)
        assert np.array_equal(rtt[acked], gr.cpu().numpy().view(np.uint64)[acked])
        got = _table(g).cpu().numpy()
        for m in range(n):
            if acked[m]:
                o = prev[peer[m]]
                oc = O.coord(oo, list(o[:8]), o[8], o[9], o[10])
                out = O.Coord()
                assert L.orc_client_update(C.byref(clients[m]), r % peers, C.byref(oc), int(rtt[m]),
                                           C.byref(O.rng(SEED, m, r)), C.byref(out)) == 0
            c = clients[m].coord
            exp = np.array(list(c.portion[:8]) + [c.error, c.adjustment, c.height])
            np.testing.assert_array_equal(got[m, :11].view(np.uint64), exp.view(np.uint64), err_msg=f"r{r} m{m}")
    for c in clients:
        L.orc_client_free(C.byref(c))
    g.close()


def test_timed_out_probes_suspect_like_oracle():
    n, peers, rounds, k = 2000, 16, 12, 2
    up_np = _up(n, 0.2, 3)
    up = torch.from_numpy(up_np).cuda()
    subj = np.arange(n, dtype=np.uint32)  # every member tracked (S = N)
    st0 = np.zeros(n, np.uint8)           # all alive
    inc0 = np.ones(n, np.uint32)
    cfg = SW.SwimConfig(n_members=n, n_subjects=n, suspicion_k=k, suspicion_min=3, suspicion_max=9)
    sw = SW.SwimState(cfg)
    sw.set_subjects(subj)
    sw.init(st0, inc0, self_incarnation=1)
    o = O.OracleSwim(0, n, n, k, sw.timeouts, subj, st0, inc0, 1)
    g = CoordinateClients(n, peers, CoordinateOptions(), seed=SEED)
    loop = ProbeLoop(g, swim=sw, wire=True)
    suspected = 0
    for r in range(rounds):
        before = o.dump()
        loop.round(r, up, now=r)
        torch.cuda.synchronize()
        peer = loop.peer.cpu().numpy()
        acked = loop.acked.cpu().numpy().astype(bool)
        msgs = []
        for m in range(n):
            if not acked[m] and up_np[m] and peer[m] != m:
                msgs.append((m, peer[m], before["incarnation"][m, peer[m]], m, SW.MSG_SUSPECT, 0))
        msgs = np.array(msgs, dtype=SW.MSG_DTYPE)
        fo, _ = o.apply(msgs, r)
        fg = loop.flags.cpu().numpy()
        want = np.zeros(n, np.int32)
        want[msgs["receiver"]] = fo
        assert np.array_equal(fg, want), r
        suspected += int(np.count_nonzero(fo & SW.F_SUSPECT))
        assert sw.tick(r) == o.tick(r)
        dg, do = sw.dump(), o.dump()
        for key in do:
            assert np.array_equal(dg[key], do[key]), f"{key} differs after round {r}"
    assert suspected > 0
    st = sw.dump()["state"]
    assert np.count_nonzero(st == SW.DEAD) > 0  # suspicion timers confirmed some dead
    sw.close()
    o.close()
    g.close()
