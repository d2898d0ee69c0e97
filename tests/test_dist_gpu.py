"""Two ranks (processes) sharing cuda:0, exchanging over gloo (host-staged): the real
HIP engine through ruserf_amd.dist.ShardedGossip must reproduce the single-context
round bit for bit.  This rehearses the driver's multi-GPU bench path (there RCCL
moves the same buffers between GPUs) on a one-GPU box."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import gossip_harness as H

pytestmark = pytest.mark.gpu
N, ROUNDS, WORLD = 3000, 8, 2


def _cfg(shard=None):
    from ruserf_amd import gossip as G
    from ruserf_amd import workload as W
    subj, acts, ml = W.churn_workload(N, ROUNDS, events_per_round=20, queries_per_round=4, seed=21)
    cfg = G.GossipConfig(n_members=N, n_subjects=len(subj), queue_cap=32, max_rumors=1 << 16,
                         event_buffer_size=128, query_buffer_size=128, slot_k=8, shard=shard)
    return cfg, subj, acts, ml


def _worker(rank, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    from ruserf_amd import workload as W
    from ruserf_amd.dist import ShardedGossip
    cfg, subj, acts, ml = _cfg()
    sg = ShardedGossip(cfg, rank, WORLD, device=0)
    sg.eng.set_subjects(subj)
    sg.eng.init_views(*W.initial_views(len(subj)))
    for t in range(ROUNDS):
        sg.round(t, ml[t], acts[t])
    torch.cuda.synchronize()
    assert sg.buckets and sg.check()
    st = H.normalize_queues(H.engine_state(sg.eng))
    q.put((rank, {k: np.asarray(v) for k, v in st.items()}))
    dist.barrier()
    sg.eng.close()
    dist.destroy_process_group()


def test_two_ranks_gloo_equal_one_context():
    from ruserf_amd import gossip as G
    from ruserf_amd import workload as W
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cfg, subj, acts, ml = _cfg()
    one = G.GossipEngine(cfg)
    one.set_subjects(subj)
    one.init_views(*W.initial_views(len(subj)))
    for t in range(ROUNDS):
        one.round(t, ml[t], acts[t])
    full = H.normalize_queues(H.engine_state(one))
    for k in full:
        assert np.array_equal(np.concatenate([got[0][k], got[1][k]]), full[k]), k
    one.close()


def _worker_rccl(port, q, exchange="buckets"):
    """ShardedGossip over RCCL ("nccl") with one rank: the exact collectives, stream
    ordering and zero-copy engine buffers of the driver's multi-GPU bench."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from ruserf_amd import workload as W
    from ruserf_amd.dist import ShardedGossip
    cfg, subj, acts, ml = _cfg()
    sg = ShardedGossip(cfg, 0, 1, device=0, exchange=exchange)
    assert not sg.stage  # RCCL moves HBM directly
    sg.eng.set_subjects(subj)
    sg.eng.init_views(*W.initial_views(len(subj)))
    for t in range(ROUNDS):
        sg.round(t, ml[t], acts[t])
    torch.cuda.synchronize()
    assert sg.buckets == (exchange == "buckets") and sg.check()
    st = H.normalize_queues(H.engine_state(sg.eng))
    q.put({k: np.asarray(v) for k, v in st.items()})
    sg.eng.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("exchange", ["buckets", "counts"])
def test_one_rank_rccl_equal_one_context(exchange):
    from ruserf_amd import gossip as G
    from ruserf_amd import workload as W
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29400 + os.getpid() % 1000
    p = ctx.Process(target=_worker_rccl, args=(port, q, exchange))
    p.start()
    got = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    cfg, subj, acts, ml = _cfg()
    one = G.GossipEngine(cfg)
    one.set_subjects(subj)
    one.init_views(*W.initial_views(len(subj)))
    for t in range(ROUNDS):
        one.round(t, ml[t], acts[t])
    full = H.normalize_queues(H.engine_state(one))
    for k in full:
        assert np.array_equal(got[k], full[k]), k
    one.close()


CFG2_N, CFG2_ROUNDS = 2_000_000, 8
CFG2_REGIME_ROUNDS = 330  # the bench's settle: queues at their steady state, the second checker pass pruning
CFG2_SAMPLE = [(0, 64), (CFG2_N // 2 - 32, 64), (CFG2_N - 64, 64)]


def _cfg2(regime=False):
    """BASELINE configs[2]'s per-GPU shard: 2M members, 4096 tracked subjects, the bench's
    gossip configuration (bench_gossip.gossip_cfg) and its 1% intent workload.  regime: the
    bench's reference queue regime (intent queue DEFAULT_QUEUE_DEPTH deep, the staggered
    checker, the ring sized so nothing expires) over CFG2_REGIME_ROUNDS rounds."""
    import bench as BB
    import bench_gossip as B
    from ruserf_amd import workload as W
    rounds = CFG2_REGIME_ROUNDS if regime else CFG2_ROUNDS
    if regime:
        cfg = B.gossip_cfg(CFG2_N, rounds, 1, queue_depth=BB.DEFAULT_QUEUE_DEPTH, ring_rounds=rounds)
    else:
        cfg = B.gossip_cfg(CFG2_N, rounds, 1)
    subj, acts, ml = W.intents_workload(CFG2_N, B.SUBJECTS, rounds, rate=0.01, seed=B.SEED,
                                        prune_frac=B.PRUNE_FRAC)
    return cfg, subj, acts, ml


def _cfg2_checker(eng, regime):
    import bench_gossip as B
    if regime:
        eng.set_checker(B.CHECK_EVERY, B.MAX_QUEUE_DEPTH, 0, B.QUEUE_DEPTH_WARNING)


def _cfg2_record(eng):
    """per-member digests, clocks, error bits and prune counts, and the sampled view rows"""
    m = eng.members()
    rec = {k: m[k].copy() for k in ["clock", "event_clock", "query_clock", "digest", "err"]}
    rec["pruned"] = eng.pruned()
    rec["expired"] = eng.expired()
    rec["merged"] = np.array([eng.merged_total()], np.uint64)
    for i, (r0, cnt) in enumerate(CFG2_SAMPLE):
        lt, st, kd, tm = eng.view(with_time=True, rows=(r0, cnt))
        rec[f"view{i}"] = np.stack([lt, st.astype(np.uint64), kd.astype(np.uint64), tm.astype(np.uint64)])
    return rec


def _worker_cfg2(port, q, regime=False):
    """The configs[2] shard through ShardedGossip on one RCCL rank (the multi-GPU code path:
    rumor-block all-reduce, bucket emission, exchange, merge from the buckets)."""
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from ruserf_amd import workload as W
    from ruserf_amd.dist import ShardedGossip
    cfg, subj, acts, ml = _cfg2(regime)
    sg = ShardedGossip(cfg, 0, 1, device=0)
    sg.eng.set_subjects(subj)
    sg.eng.init_views(*W.initial_views(len(subj)))
    _cfg2_checker(sg.eng, regime)
    for t in range(len(acts)):
        sg.round(t, ml[t], acts[t])
    torch.cuda.synchronize()
    rec = _cfg2_record(sg.eng)
    if regime:
        rec["queue_lengths"] = sg.eng.queue_lengths()[:, 0].copy()
        rec["checker"] = np.array(sum((list(v) for v in sg.eng.checker_stats().values()), []), np.uint64)
    rec["exchange_ok"] = np.array([sg.buckets and sg.check()])
    sg.eng.close()
    dist.destroy_process_group()
    q.put(rec)


def test_configs2_shard_regime_rccl_equal_one_context():
    """BASELINE configs[2]'s per-GPU shard (2M members x 4096 subjects) in the bench's reference
    queue regime -- the intent queue 8 704 deep (packed 8-B tail items, 12-B view entries: the
    regime fits one MI355X at 2M members), each member's QueueChecker pruning to 4096 every
    150 rounds on its own phase, 330 rounds so the second pass prunes queues of 4-8k items --
    through the multi-GPU code path on one RCCL rank, equal to the single-context round: every
    member's clocks, digest, error bits, prunes and expiries, its intent queue length, the
    checker's counts, the records merged and sampled view rows; nothing dropped between ticks,
    nothing expired.  (The rank runs first, in its own process, then the single context.)"""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from ruserf_amd import gossip as G
    from ruserf_amd import workload as W
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + os.getpid() % 200
    p = ctx.Process(target=_worker_cfg2, args=(port, q, True))
    p.start()
    got = q.get(timeout=900)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert bool(got.pop("exchange_ok")[0])
    cfg, subj, acts, ml = _cfg2(True)
    one = G.GossipEngine(cfg)
    one.set_subjects(subj)
    one.init_views(*W.initial_views(len(subj)))
    _cfg2_checker(one, True)
    for t in range(len(acts)):
        one.round(t, ml[t], acts[t])
    exp = _cfg2_record(one)
    exp["queue_lengths"] = one.queue_lengths()[:, 0].copy()
    exp["checker"] = np.array(sum((list(v) for v in one.checker_stats().values()), []), np.uint64)
    one.close()
    for k in exp:
        assert np.array_equal(got[k], exp[k]), k
    ql = exp["queue_lengths"].astype(np.int64)
    assert ql.mean() > 4096 and int(ql.max()) > 7000, (ql.mean(), ql.max())  # the regime's occupancy
    assert int(exp["pruned"].sum()) == 0 and int(exp["expired"].sum()) == 0
    assert np.all(exp["err"] == 0)
    assert int(exp["checker"][6]) > 0  # the ticks pruned


def test_configs2_shard_rccl_equal_one_context():
    """BASELINE configs[2] at its per-GPU shard size (2M members x 4096 subjects, 8 rounds):
    the multi-GPU code path on one RCCL rank must equal the single-context round -- every
    member's clocks, digest (of every delivery), error bits and queue prunes, the records
    merged, and sampled view rows -- with no bucket over capacity (exchange_ok).  The two
    runs hold ~150 GB each and run one after the other (the rank first, in its own process)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from ruserf_amd import gossip as G
    from ruserf_amd import workload as W
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29300 + os.getpid() % 1000
    p = ctx.Process(target=_worker_cfg2, args=(port, q))
    p.start()
    got = q.get(timeout=600)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert bool(got.pop("exchange_ok")[0])
    cfg, subj, acts, ml = _cfg2()
    one = G.GossipEngine(cfg)
    one.set_subjects(subj)
    one.init_views(*W.initial_views(len(subj)))
    for t in range(CFG2_ROUNDS):
        one.round(t, ml[t], acts[t])
    exp = _cfg2_record(one)
    one.close()
    assert int(exp["merged"][0]) > CFG2_N  # the rounds carried traffic
    for k in exp:
        assert np.array_equal(got[k], exp[k]), k
