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
