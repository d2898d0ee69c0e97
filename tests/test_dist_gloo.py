"""world_size-2 gloo test (CPU) of the multi-GPU round driver (ruserf_amd.dist):
rumor-block all-reduce, record counts exchange and the all-to-all routing that
must deliver each shard its records concatenated in source-rank order.  The
HIP engine is replaced by a CPU stand-in that only produces/consumes records
(the engine's split API itself is checked on the GPU in test_gossip_gpu.py)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N, WORLD, ROUNDS = 64, 2, 3


class FakeEngine:
    def __init__(self, rank):
        self.rank = rank
        self.per = N // WORLD
        self.block = torch.zeros(WORLD * 4 * 3, dtype=torch.int64)
        self.send_t = torch.zeros(4096, dtype=torch.int64)
        self.received = []
        self.t = 0

    def round_begin(self, t, ml, acts):
        self.t = t
        self.block.zero_()
        # entries [rank*4, rank*4+4) are owned by this shard
        for j in range(4):
            self.block[(self.rank * 4 + j) * 3] = 1000 * t + 10 * self.rank + j

    def round_emit(self, world):
        rng = np.random.default_rng(100 * self.t + self.rank)
        recs = []
        for local in range(self.per):
            sender = self.rank * self.per + local
            for pos in range(3):
                recv = int(rng.integers(0, N))
                recs.append((recv, (sender << 8) | pos))
        recs.sort(key=lambda x: x[0])  # stable by receiver: sender-major order kept
        packed = np.array([(r << 32) | v for r, v in recs], dtype=np.int64)
        self.send_t[: len(packed)] = torch.from_numpy(packed)
        counts = np.zeros(world, dtype=np.uint64)
        for r, _ in recs:
            counts[r // self.per] += 1
        return counts


class FakeBuffers:
    def __init__(self, eng):
        self.eng = eng
        self.send = eng.send_t
        self.recv = torch.zeros(4096, dtype=torch.int64)

    def rumor_block(self):
        return self.eng.block

    def merge(self, n, run_counts=None):
        self.eng.received.append(self.recv[:n].clone().numpy())


def _worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    from ruserf_amd.dist import ShardedGossip
    from ruserf_amd.gossip import GossipConfig
    eng = FakeEngine(rank)
    sg = ShardedGossip(GossipConfig(n_members=N, n_subjects=4), rank, WORLD, engine=eng, buffers=FakeBuffers(eng))
    out = []
    for t in range(ROUNDS):
        sg.round(t)
        blk = eng.block.numpy().copy()
        out.append((blk, eng.received[-1]))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def expected_for(rank, t):
    per = N // WORLD
    recs = []
    for src in range(WORLD):
        rng = np.random.default_rng(100 * t + src)
        for local in range(per):
            sender = src * per + local
            for pos in range(3):
                recv = int(rng.integers(0, N))
                if recv // per == rank:
                    recs.append((recv, (sender << 8) | pos))
    # concatenation in source-rank order of per-source receiver-sorted chunks
    out = []
    for src in range(WORLD):
        chunk = [r for r in recs if ((r[1] >> 8) // per) == src]
        chunk.sort(key=lambda x: x[0])
        out += chunk
    return np.array([(r << 32) | v for r, v in out], dtype=np.int64)


def test_sharded_round_routing_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 2000)
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(WORLD):
        for t, (blk, recv) in enumerate(res[rank]):
            want = np.zeros(WORLD * 4 * 3, dtype=np.int64)
            for src in range(WORLD):
                for j in range(4):
                    want[(src * 4 + j) * 3] = 1000 * t + 10 * src + j
            assert np.array_equal(blk, want)
            assert np.array_equal(recv, expected_for(rank, t))
            # stable sort by receiver of the concatenation = canonical (receiver, sender, pos)
            keys = recv >> 32
            order = np.argsort(keys, kind="stable")
            senders = (recv[order] & 0xFFFFFFFF) >> 8
            for rcv in np.unique(keys):
                sel = senders[keys[order] == rcv]
                assert np.all(np.diff(sel) >= 0)


class FakeBucketBuffers:
    """Bucket exchange stand-in: every rank fills bucket w with (src, w, i) words; the
    merge records what arrived (must be each source's bucket for this rank, in
    source-rank order)."""

    def __init__(self, rank, world, words=16):
        self.rank, self.world, self.words, self.bucket_words, self.buckets = rank, world, words, words, True
        self.block = torch.zeros(12, dtype=torch.int64)
        self.send = torch.zeros(world * words, dtype=torch.int32)
        self.recv = torch.zeros(world * words, dtype=torch.int32)
        self.received = []

    def rumor_block(self):
        return self.block

    def emit(self):
        for w in range(self.world):
            self.send[w * self.words:(w + 1) * self.words] = torch.tensor(
                [1000 * self.rank + 100 * w + i for i in range(self.words)], dtype=torch.int32)

    def merge(self, n_recv=None, run_counts=None):
        self.received.append(self.recv.clone().numpy())

    def ok(self):
        return True


class FakeBeginEngine:
    def round_begin(self, t, ml, acts):
        pass


def _worker_buckets(rank, port, q, world):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ruserf_amd.dist import ShardedGossip
    from ruserf_amd.gossip import GossipConfig
    buf = FakeBucketBuffers(rank, world)
    sg = ShardedGossip(GossipConfig(n_members=N * 3, n_subjects=4), rank, world, engine=FakeBeginEngine(), buffers=buf)
    assert sg.buckets
    sg.round(0)
    assert sg.check()
    q.put((rank, buf.received[-1]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_round_buckets_gloo(world):
    """The bucket exchange: grouped point-to-point sends/receives, no host-side counts; rank r
    receives bucket r of every other source, in source-rank order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + world * 2000 + (os.getpid() % 2000)
    procs = [ctx.Process(target=_worker_buckets, args=(r, port, q, world)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(world):
        # the self slot is never filled: the merge reads the rank's own bucket from its send buffer
        want = np.concatenate([[1000 * src + 100 * rank + i if src != rank else 0 for i in range(16)]
                               for src in range(world)])
        assert np.array_equal(res[rank], want.astype(np.int32))
