"""GPU parity: the HIP Vivaldi kernels against the CPU oracle, bit-exact.

North-star tolerance for float64 coordinates is 1e-9 relative; the kernels are
built with -ffp-contract=off and are expected to be BIT-EXACT, which these
tests assert (ATOL = RTOL = 0)."""
import ctypes as C
import math

import numpy as np
import pytest

import oracle_ffi as O
from ruserf_amd import Coordinate, CoordinateClients, CoordinateError, CoordinateOptions

pytestmark = pytest.mark.gpu
L = O.lib()
SEED = 0x5EED5EED


def oracle_pop(n, peers, opts, seed=SEED):
    p = O.VivaldiPop()
    oo = O.default_opts(dimensionality=opts.dimensionality, height_min=opts.height_min,
                        latency_filter_size=opts.latency_filter_size,
                        adjustment_window_size=opts.adjustment_window_size)
    assert L.orc_vivaldi_pop_init(C.byref(p), n, peers, C.byref(oo), seed) == 0
    return p


def oracle_rows(p):
    return O.arr(p.rows_cur, p.n * p.row_stride, np.float64).reshape(p.n, p.row_stride).copy()


@pytest.mark.parametrize("n,peers,rounds,dim,F", [(1000, 16, 60, 8, 3), (257, 5, 25, 3, 3),
                                                  (300, 4, 20, 8, 5)])
def test_population_rounds_bit_exact(n, peers, rounds, dim, F):
    opts = CoordinateOptions(dimensionality=dim, latency_filter_size=F)
    g = CoordinateClients(n, peers, opts, seed=SEED)
    p = oracle_pop(n, peers, opts)
    for t in range(rounds):
        g.round(t)
    L.orc_vivaldi_pop_rounds(C.byref(p), 0, rounds, 8)
    got, exp = g.get_rows(), oracle_rows(p)
    assert np.all(np.isfinite(got))
    np.testing.assert_array_equal(got.view(np.uint64), exp.view(np.uint64))
    assert g.stats()["resets"] == p.resets
    L.orc_vivaldi_pop_free(C.byref(p))
    g.close()


def test_population_large_bit_exact():
    # 200k members x 4 rounds (the oracle needs a few seconds on 8 threads)
    n, peers, rounds = 200_000, 16, 4
    opts = CoordinateOptions()
    g = CoordinateClients(n, peers, opts, seed=SEED ^ 0xABC)
    p = oracle_pop(n, peers, opts, seed=SEED ^ 0xABC)
    for t in range(rounds):
        g.round(t)
    L.orc_vivaldi_pop_rounds(C.byref(p), 0, rounds, 8)
    np.testing.assert_array_equal(g.get_rows().view(np.uint64), oracle_rows(p).view(np.uint64))
    L.orc_vivaldi_pop_free(C.byref(p))
    g.close()


def test_round_is_deterministic_and_converges():
    n = 1000
    a = CoordinateClients(n, 16, seed=SEED)
    b = CoordinateClients(n, 16, seed=SEED)
    for t in range(200):
        a.round(t)
        b.round(t)
    np.testing.assert_array_equal(a.get_rows(), b.get_rows())
    # estimate_rtt vs ground truth: median relative error over random pairs
    rng = np.random.default_rng(1)
    i = rng.integers(0, n, 4000, dtype=np.uint32)
    j = rng.integers(0, n, 4000, dtype=np.uint32)
    keep = i != j
    est = a.distance_to(i[keep], j[keep]).astype(np.float64)
    true = np.array([a.true_rtt_ns(int(x), int(y)) for x, y in zip(i[keep], j[keep])], dtype=np.float64)
    med = np.median(np.abs(est - true) / true)
    assert med < 0.25, med


def test_estimate_rtt_matches_oracle():
    n = 2000
    g = CoordinateClients(n, 8, seed=SEED)
    for t in range(10):
        g.round(t)
    rows = g.get_rows()
    rng = np.random.default_rng(2)
    a = rng.integers(0, n, 5000, dtype=np.uint32)
    b = rng.integers(0, n, 5000, dtype=np.uint32)
    got = g.distance_to(a, b)
    opts = O.default_opts()
    for k in range(0, 5000, 7):
        ca = O.coord(opts, list(rows[a[k], :8]), rows[a[k], 8], rows[a[k], 9], rows[a[k], 10])
        cb = O.coord(opts, list(rows[b[k], :8]), rows[b[k], 8], rows[b[k], 9], rows[b[k], 10])
        assert got[k] == L.orc_coord_distance_ns(C.byref(ca), C.byref(cb))


def test_update_batch_matches_oracle_clients():
    """Batched CoordinateClient::update with explicit `other` coordinates, including
    every error path, against one oracle client per member."""
    n, slots, dim = 64, 4, 8
    opts = CoordinateOptions()
    g = CoordinateClients(n, slots, opts, seed=SEED)
    oo = O.default_opts()
    clients = []
    for m in range(n):
        c = O.Client()
        assert L.orc_client_init(C.byref(c), C.byref(oo), slots) == 0
        clients.append(c)
    rng = np.random.default_rng(3)
    for rnd in range(30):
        members = rng.permutation(n)[:40].astype(np.uint32)
        slot = rng.integers(0, slots, 40).astype(np.uint32)
        others, rtts = [], []
        for i in range(40):
            o = Coordinate(rng.normal(0, 0.02, dim), float(rng.uniform(0, 1.5)), float(rng.normal(0, 1e-3)),
                           float(rng.uniform(1e-5, 1e-3)))
            kind = rng.integers(0, 20)
            if kind == 0:
                o.portion[1] = math.nan
            elif kind == 1:
                o = Coordinate(np.zeros(3), 1.5, 0.0, 1e-5)
            rtt = int(rng.integers(0, 200_000_000))
            if kind == 2:
                rtt = 10_000_000_001
            if kind == 3:
                rtt = 10_000_000_000  # equality is accepted (rtt > MAX_RTT rejects)
            if kind == 4:
                rtt = 0
            others.append(o)
            rtts.append(rtt)
        status, rows = g.update_batch(members, slot, others, rtts, round_=rnd)
        for i in range(40):
            m = int(members[i])
            oc = O.coord(oo, list(others[i].portion), others[i].error, others[i].adjustment, others[i].height)
            r = O.rng(SEED, m, rnd)
            out = O.Coord()
            e = L.orc_client_update(C.byref(clients[m]), int(slot[i]), C.byref(oc), rtts[i], C.byref(r), C.byref(out))
            assert status[i] == e, (rnd, i)
            c = clients[m].coord
            exp = np.array(list(c.portion[:8]) + [c.error, c.adjustment, c.height])
            np.testing.assert_array_equal(rows[i, :11].view(np.uint64), exp.view(np.uint64))
    for c in clients:
        L.orc_client_free(C.byref(c))
    g.close()


def test_client_kats_through_engine(kats):
    k = kats["coordinate"]
    opts = CoordinateOptions(dimensionality=3)
    g = CoordinateClients(4, 2, opts)
    other = Coordinate(np.array(k["client_update"]["other_portion"]), 1.5, 0.0, 10e-6)
    c = g.update(0, 0, other, k["client_update"]["rtt_ns"])
    assert c.portion[2] < 0.0  # coordinate.rs:904
    c.portion[2] = 99.0
    g.set_coordinate(0, c)
    assert g.get_coordinate(0).portion[2] == 99.0
    # invalid pings (coordinate.rs:913-938)
    g.set_coordinate(1, Coordinate.with_options(opts))
    g.set_coordinate(2, other)
    d0 = g.distance_to([1], [2])[0]
    for ns in k["client_invalid_in_ping_values"]["rtt_ns"]:
        with pytest.raises(CoordinateError) as ei:
            g.update(1, 0, other, ns)
        assert ei.value.code == CoordinateError.INVALID_RTT
        assert g.distance_to([1], [2])[0] == d0
    # nan defense (1035-1067)
    bad = Coordinate(np.array([math.nan, 0.0, 0.0]), 1.5, 0.0, 10e-6)
    with pytest.raises(CoordinateError) as ei:
        g.update(3, 0, bad, 250_000_000)
    assert ei.value.code == CoordinateError.INVALID_COORDINATE
    with pytest.raises(CoordinateError) as ei:
        g.set_coordinate(3, Coordinate(np.zeros(6), 1.5, 0.0, 1e-5))
    assert ei.value.code == CoordinateError.DIMENSIONALITY_MISMATCH
    # distance_to with height_min 0 (940-954)
    h0 = CoordinateClients(2, 1, CoordinateOptions(dimensionality=3, height_min=0.0))
    h0.set_coordinate(1, Coordinate(np.array([0.0, 0.0, 12.345]), 1.5, 0.0, 0.0))
    assert h0.distance_to([0], [1])[0] == k["client_distance_to"]["expect_ns"]
    g.close()
    h0.close()


def test_gen_probes_match_oracle():
    """The synthetic network's probes (the bench's resident inputs) equal the oracle's."""
    import torch
    n, peers = 5000, 16
    g = CoordinateClients(n, peers, seed=SEED)
    nbr = np.empty(n * peers, dtype=np.uint32)
    L.orc_gen_neighbors(SEED, n, peers, nbr.ctypes.data_as(O.P32))
    peer = torch.empty(n, dtype=torch.int32, device="cuda")
    rtt = torch.empty(n, dtype=torch.int64, device="cuda")
    for r in (0, 1, 17, 1000):
        g.gen_probes(r, peer.data_ptr(), rtt.data_ptr())
        torch.cuda.synchronize()
        gp = peer.cpu().numpy().view(np.uint32)
        gr = rtt.cpu().numpy().view(np.uint64)
        for m in range(0, n, 13):
            slot, ns = C.c_uint32(), C.c_uint64()
            L.orc_vivaldi_probe(SEED, n, peers, nbr.ctypes.data_as(O.P32), m, r, C.byref(slot), C.byref(ns))
            assert slot.value == r % peers
            assert gp[m] == nbr[m * peers + slot.value], (r, m)
            assert gr[m] == ns.value, (r, m)
    g.close()


def test_observe_explicit_probes_matches_oracle_clients():
    """rsf_vivaldi_observe with caller-provided, device-resident (peer, rtt) inputs —
    including invalid RTTs and out-of-range peers — against one oracle client per
    member fed the same peer coordinates (previous-round snapshot)."""
    import torch
    n, slots = 96, 4
    g = CoordinateClients(n, slots, seed=SEED)
    oo = O.default_opts()
    clients = []
    for m in range(n):
        c = O.Client()
        assert L.orc_client_init(C.byref(c), C.byref(oo), slots) == 0
        clients.append(c)
    rng = np.random.default_rng(9)
    stride = g.stride
    for rnd in range(24):
        snap = g.get_rows()  # previous-round table (= the oracle clients' coordinates)
        peer = rng.integers(0, n, n).astype(np.uint32)
        peer[peer == np.arange(n)] = (peer[peer == np.arange(n)] + 1) % n
        rtt = rng.integers(1_000_000, 80_000_000, n).astype(np.uint64)
        kind = rng.integers(0, 16, n)
        rtt[kind == 0] = 10_000_000_001  # InvalidRTT
        rtt[kind == 1] = 10_000_000_000  # equality accepted
        peer[kind == 2] = n + 5          # out of range -> RSF_ERR_ARG
        dp = torch.from_numpy(peer.view(np.int32)).cuda()
        dr = torch.from_numpy(rtt.view(np.int64)).cuda()
        ds = torch.empty(n, dtype=torch.int32, device="cuda")
        slot = rnd % slots
        g.observe(slot, dp.data_ptr(), dr.data_ptr(), ds.data_ptr(), round_=rnd)
        torch.cuda.synchronize()
        status = ds.cpu().numpy()
        rows = g.get_rows()
        for m in range(n):
            if peer[m] >= n:
                assert status[m] == -1  # RSF_ERR_ARG
                np.testing.assert_array_equal(rows[m].view(np.uint64), snap[m].view(np.uint64))
                continue
            o = snap[peer[m]]
            oc = O.coord(oo, list(o[:8]), o[8], o[9], o[10])
            out = O.Coord()
            e = L.orc_client_update(C.byref(clients[m]), slot, C.byref(oc), int(rtt[m]), C.byref(O.rng(SEED, m, rnd)),
                                    C.byref(out))
            assert status[m] == e, (rnd, m)
            c = clients[m].coord
            exp = np.array(list(c.portion[:8]) + [c.error, c.adjustment, c.height])
            np.testing.assert_array_equal(rows[m, :11].view(np.uint64), exp.view(np.uint64))
        assert stride == rows.shape[1]
    for c in clients:
        L.orc_client_free(C.byref(c))
    g.close()


class _DevArray:
    """zero-copy torch view of engine-owned HBM (test hook)"""

    def __init__(self, ptr, n, typestr="<f8"):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (int(ptr), False),
                                         "version": 3, "strides": None}


def _table(g):
    import torch
    ptr, stride = g.table_ptr()
    return torch.as_tensor(_DevArray(ptr, g.n * stride), device="cuda").view(g.n, stride)


def test_forget_node_matches_oracle_clients():
    """CoordinateClient::forget_node (coordinate.rs:455-457) drops a peer's latency-filter
    samples: updates before and after a forget, against oracle clients that forget the
    same (member, slot) at the same point (the reference's test_client_latency_filter,
    coordinate.rs:1024-1032, through the whole update)."""
    n, slots = 48, 3
    g = CoordinateClients(n, slots, CoordinateOptions(), seed=SEED)
    oo = O.default_opts()
    clients = []
    for m in range(n):
        c = O.Client()
        assert L.orc_client_init(C.byref(c), C.byref(oo), slots) == 0
        clients.append(c)
    rng = np.random.default_rng(13)
    for rnd in range(24):
        if rnd % 4 == 3:  # forget a few (member, slot) pairs
            for m, s in zip(rng.integers(0, n, 10), rng.integers(0, slots, 10)):
                g.forget_node(int(m), int(s))
                L.orc_client_forget_node(C.byref(clients[int(m)]), int(s))
        members = rng.permutation(n)[:32].astype(np.uint32)
        slot = rng.integers(0, slots, 32).astype(np.uint32)
        others = [Coordinate(rng.normal(0, 0.02, 8), float(rng.uniform(0.1, 1.5)), float(rng.normal(0, 1e-3)),
                             float(rng.uniform(1e-5, 1e-3))) for _ in range(32)]
        rtts = [int(x) for x in rng.integers(1_000_000, 300_000_000, 32)]
        status, rows = g.update_batch(members, slot, others, rtts, round_=rnd)
        for i in range(32):
            m = int(members[i])
            o = others[i]
            oc = O.coord(oo, list(o.portion), o.error, o.adjustment, o.height)
            out = O.Coord()
            e = L.orc_client_update(C.byref(clients[m]), int(slot[i]), C.byref(oc), rtts[i],
                                    C.byref(O.rng(SEED, m, rnd)), C.byref(out))
            assert status[i] == e == 0
            c = clients[m].coord
            exp = np.array(list(c.portion[:8]) + [c.error, c.adjustment, c.height])
            np.testing.assert_array_equal(rows[i, :11].view(np.uint64), exp.view(np.uint64))
    for c in clients:
        L.orc_client_free(C.byref(c))
    g.close()


def test_nan_defense_reset_through_engine():
    """test_client_nan_defense (coordinate.rs:1061-1066): a poisoned internal coordinate
    is reset by the next update (stats().resets == 1) -- the engine's table poisoned in
    HBM, the oracle client's in memory, same update, same bits."""
    import torch
    opts = CoordinateOptions(dimensionality=3)
    g = CoordinateClients(2, 1, opts, seed=SEED)
    t = _table(g)
    t[0, 0] = float("nan")
    torch.cuda.synchronize()
    other = Coordinate.with_options(opts)
    c = g.update(0, 0, other, 250_000_000)
    assert c.is_valid() and g.stats()["resets"] == 1
    oo = O.default_opts(dimensionality=3)
    cl = O.Client()
    assert L.orc_client_init(C.byref(cl), C.byref(oo), 1) == 0
    cl.coord.portion[0] = float("nan")
    out = O.Coord()
    assert L.orc_client_update(C.byref(cl), 0, C.byref(O.coord(oo, [0.0, 0.0, 0.0])), 250_000_000,
                               C.byref(O.rng(SEED, 0, 0)), C.byref(out)) == 0
    assert cl.resets == 1
    exp = np.array(list(cl.coord.portion[:3]) + [cl.coord.error, cl.coord.adjustment, cl.coord.height])
    np.testing.assert_array_equal(g.get_rows(0, 1)[0, :6].view(np.uint64), exp.view(np.uint64))
    L.orc_client_free(C.byref(cl))
    g.close()


def test_64m_population_properties_and_sampled_parity():
    """BASELINE configs[4] at full size: 64M members, D=8, F=3, W=20, 16 neighbours.
    Four rounds from device-resident probes; a 10k-member sample is checked BIT-EXACT
    every round against oracle clients fed the same probe and the peer's row of the
    previous-round table; the whole table stays finite with no resets; a second
    context with the same seed produces the same table."""
    import torch
    n, peers, rounds, ns = 64_000_000, 16, 4, 10_000
    rng = np.random.default_rng(64)
    sample = np.sort(rng.choice(n, ns, replace=False)).astype(np.int64)
    sidx = torch.from_numpy(sample).cuda()
    oo = O.default_opts()
    clients = []
    for _ in range(ns):
        c = O.Client()
        assert L.orc_client_init(C.byref(c), C.byref(oo), peers) == 0
        clients.append(c)
    g = CoordinateClients(n, peers, CoordinateOptions(), seed=SEED)
    peer = torch.empty(n, dtype=torch.int32, device="cuda")
    rtt = torch.empty(n, dtype=torch.int64, device="cuda")
    for r in range(rounds):
        g.gen_probes(r, peer.data_ptr(), rtt.data_ptr())
        g.sync()  # the engine runs on its own stream; torch reads the probes next
        prev = _table(g)
        sp = peer[sidx].long()
        prow = prev[sp].cpu().numpy()
        srtt = rtt[sidx].cpu().numpy().view(np.uint64)
        g.observe(r % peers, peer.data_ptr(), rtt.data_ptr(), None, r)
        torch.cuda.synchronize()
        got = _table(g)[sidx].cpu().numpy()
        for i in range(ns):
            m = int(sample[i])
            o = prow[i]
            oc = O.coord(oo, list(o[:8]), o[8], o[9], o[10])
            out = O.Coord()
            assert L.orc_client_update(C.byref(clients[i]), r % peers, C.byref(oc), int(srtt[i]),
                                       C.byref(O.rng(SEED, m, r)), C.byref(out)) == 0
            c = clients[i].coord
            exp = np.array(list(c.portion[:8]) + [c.error, c.adjustment, c.height])
            np.testing.assert_array_equal(got[i, :11].view(np.uint64), exp.view(np.uint64), err_msg=f"r{r} m{m}")
    full = _table(g)[:, :11]
    assert bool(torch.isfinite(full).all())
    assert g.stats()["resets"] == 0
    h = CoordinateClients(n, peers, CoordinateOptions(), seed=SEED)
    for r in range(rounds):
        h.gen_probes(r, peer.data_ptr(), rtt.data_ptr())
        h.observe(r % peers, peer.data_ptr(), rtt.data_ptr(), None, r)
    torch.cuda.synchronize()
    assert torch.equal(_table(h)[:, :11].view(torch.int64), full.view(torch.int64))
    for c in clients:
        L.orc_client_free(C.byref(c))
    g.close()
    h.close()


def test_configs0_c1_gpu_matches_cpu_path():
    """configs[0]'s 1k-node run (bench.c1_leg, 300 rounds): the HIP engine's coordinates are
    bit-identical to the CPU path's after every update."""
    import bench
    r = bench.c1_leg(rounds=300)
    assert r["gpu_bit_exact"] and r["median_rel_rtt_error_all_pairs"] < 0.2
