"""Sharded Vivaldi rounds: two ranks (processes) sharing cuda:0 over gloo (host-staged)
run ruserf_amd.dist.ShardedVivaldi -- each round fetches only the rows of its members'
remote peers from their owners (request / reply all-to-all) -- and must
reproduce one context that holds every member, bit for bit (rows, and the latency
filters / adjustment windows through the rows they produce)."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
N, ROUNDS, SEED = 24_000, 14, 0x5EED


def _worker(rank, world, port, q, presend=False, chunks=1):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ruserf_amd import CoordinateClients, CoordinateOptions
    from ruserf_amd.dist import ShardedVivaldi
    per = N // world
    lo, hi = rank * per, (rank + 1) * per
    g = CoordinateClients(N, 16, CoordinateOptions(), seed=SEED, device=0, shard=(lo, hi))
    g.set_stream(torch.cuda.current_stream().cuda_stream)
    sv = ShardedVivaldi(g, rank, world)
    assert sv.stage
    # every round's probes up front (the next round's requests can go out during a round)
    peer = torch.empty((ROUNDS, per), dtype=torch.int32, device="cuda")
    rtt = torch.empty((ROUNDS, per), dtype=torch.int64, device="cuda")
    remote = 0
    for r in range(ROUNDS):
        g.gen_probes(r, peer[r].data_ptr(), rtt[r].data_ptr())
        p = peer[r].cpu().numpy()
        remote += int(np.count_nonzero((p < lo) | (p >= hi)))
    for r in range(ROUNDS):
        nxt = peer[r + 1].data_ptr() if presend and r + 1 < ROUNDS else None
        sv.round(r, peer[r].data_ptr(), rtt[r].data_ptr(), next_peer_ptr=nxt, chunks=chunks)
    torch.cuda.synchronize()
    ok = sv.check()
    rows = g.get_rows(lo, per)
    q.put((rank, rows, ok, remote, g.stats()["resets"]))
    dist.barrier()
    g.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,presend,chunks", [(2, False, 1), (2, True, 1), (2, False, 4), (2, False, 7)])
def test_sharded_vivaldi_equals_one_context(world, presend, chunks):
    """presend: round r + 1's requests built and exchanged on a side stream during round r
    (ShardedVivaldi.presend); chunks > 1: the round pipelined by member chunks, chunk i
    observed while chunk i + 1's rows are exchanged on a side stream (round_chunked; 7 chunks
    leave the last one short).  The result is the same bit for bit."""
    from ruserf_amd import CoordinateClients, CoordinateOptions
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + os.getpid() % 1000 + (7 if presend else 0) + 13 * chunks
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, presend, chunks)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        rank, rows, ok, remote, resets = q.get(timeout=300)
        got[rank] = (rows, ok, remote, resets)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    one = CoordinateClients(N, 16, CoordinateOptions(), seed=SEED, device=0)
    for r in range(ROUNDS):
        one.round(r)
    one.sync()
    full = one.get_rows()
    resets = one.stats()["resets"]
    one.close()
    for rank in range(world):
        assert got[rank][1], f"rank {rank}: exchange overflow / misrouted request"
        # most probes cross shards: the exchange is exercised, not bypassed
        assert got[rank][2] > ROUNDS * (N // world) // 4
    sharded = np.concatenate([got[r][0] for r in range(world)])
    assert np.array_equal(sharded.view(np.uint64), full.view(np.uint64))
    assert sum(got[r][3] for r in range(world)) == resets


def _worker_allgather(rank, world, port, R, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ruserf_amd import CoordinateClients, CoordinateOptions
    from ruserf_amd.dist import VivaldiTableRefresh
    per = N // world
    lo, hi = rank * per, (rank + 1) * per
    g = CoordinateClients(N, 16, CoordinateOptions(), seed=SEED, device=0, shard=(lo, hi))
    g.set_stream(torch.cuda.current_stream().cuda_stream)
    ref = VivaldiTableRefresh(g, rank, world, R)
    peer = torch.empty(per, dtype=torch.int32, device="cuda")
    rtt = torch.empty(per, dtype=torch.int64, device="cuda")
    for r in range(ROUNDS):
        g.gen_probes(r, peer.data_ptr(), rtt.data_ptr())
        read_ptr = g.table_ptr()[0]
        g.observe(r % 16, peer.data_ptr(), rtt.data_ptr(), None, r)
        ref.after_round(r, read_ptr)
    torch.cuda.synchronize()
    q.put((rank, g.get_rows(lo, per)))
    dist.barrier()
    g.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("R", [8, 1, 3])
def test_allgather_refresh_matches_stale_oracle(R):
    """The all-gather refresh of the coordinate table (dist.VivaldiTableRefresh, SURVEY §8(d)
    C5: R = 1 and R = 8; an odd R as well) over two ranks sharing cuda:0 (gloo, host-staged):
    a member reads its own shard's peers from the previous round and other shards' peers as
    of the last refresh.  Bit-exact against the oracle's rounds with exactly that staleness
    (orc_vivaldi_pop_rounds_stale)."""
    import ctypes as C

    import oracle_ffi as O
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + (os.getpid() + R) % 1000
    procs = [ctx.Process(target=_worker_allgather, args=(r, world, port, R, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        rank, rows = q.get(timeout=300)
        got[rank] = rows
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    L = O.lib()
    pop = O.VivaldiPop()
    oo = O.default_opts()
    assert L.orc_vivaldi_pop_init(C.byref(pop), N, 16, C.byref(oo), SEED) == 0
    stale = O.arr(pop.rows_cur, N * pop.row_stride, np.float64).copy()
    assert L.orc_vivaldi_pop_rounds_stale(C.byref(pop), 0, ROUNDS, 8, stale.ctypes.data_as(C.POINTER(C.c_double)),
                                          N // world, R) == 0
    exp = O.arr(pop.rows_cur, N * pop.row_stride, np.float64).reshape(N, pop.row_stride).copy()
    sharded = np.concatenate([got[r] for r in range(world)])
    assert np.array_equal(sharded.view(np.uint64), exp.view(np.uint64))
    if R > 1:  # the staleness matters: the fresh-table rounds differ
        L.orc_vivaldi_pop_free(C.byref(pop))
        assert L.orc_vivaldi_pop_init(C.byref(pop), N, 16, C.byref(oo), SEED) == 0
        L.orc_vivaldi_pop_rounds(C.byref(pop), 0, ROUNDS, 8)
        fresh = O.arr(pop.rows_cur, N * pop.row_stride, np.float64).reshape(N, pop.row_stride)
        assert not np.array_equal(fresh.view(np.uint64), exp.view(np.uint64))
    L.orc_vivaldi_pop_free(C.byref(pop))
