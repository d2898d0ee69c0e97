"""Multi-GPU gossip rounds: one process per GPU, members sharded by contiguous
id range, RCCL collectives through torch.distributed.

Per round:
  1. round_begin   — each shard runs memberlist transitions, refutations and
                     originations for ITS members; every rumor-table entry of
                     the round is owned by exactly one shard
  2. all-reduce    — SUM of the round's rumor block (non-owners hold zeros), so
                     every shard can resolve every rumor id it will receive
  3. exchange, by default through fixed-capacity BUCKETS (no host synchronisation):
       round_emit_buckets  — peer draw, stable sort of the (sender, peer) groups by
                             global receiver, emission straight into one bucket per
                             destination shard
       exchange            — bucket w of every rank goes to slot (source rank) of rank
                             w's receive buffer: grouped point-to-point sends/receives
                             (one RCCL group), every pair except the rank's own bucket,
                             which the merge reads from the send buffer in place
       round_merge_buckets — per receiver, its groups of every source in source-rank
                             order = the canonical (receiver; sender, position) order,
                             merged straight from the received buckets
     Bucket overflow (a destination receiving far more groups than the uniform share)
     is recorded on the device and checked by `check()`.
     The counts exchange (world > 8, or exchange="counts"): round_emit compacts the
     records into one receiver-sorted stream, the counts go through an all-to-all and
     the host, then the records, and round_merge_runs rebuilds the canonical order.

The driver is generic over the engine object (`GossipEngine` on HIP; the gloo
tests substitute a CPU stand-in that exercises only the routing).

Vivaldi rounds (ShardedVivaldi): each shard holds the whole coordinate table but
updates only its own rows; a round fetches just the rows of its members' remote
peers from their owners (request all-to-all, owners copy the rows, reply all-to-all,
rows written in place), then observes -- the targeted exchange of SURVEY §8(e) in
place of an all-gather of the table.
"""
import dataclasses

import numpy as np
import torch
import torch.distributed as dist

from .gossip import GossipConfig, GossipEngine

MAX_BUCKET_WORLD = 8  # kMaxRuns in csrc/gossip.hip


class CudaArray:
    """Zero-copy view of engine-owned HBM for torch (RCCL) collectives."""

    def __init__(self, ptr, n, typestr):
        self.__cuda_array_interface__ = {"shape": (int(n),), "typestr": typestr, "data": (int(ptr), False),
                                         "version": 3, "strides": None}


def hbm_tensor(ptr, n, typestr="<i8"):
    if n == 0:
        return torch.empty(0, dtype=torch.int64, device="cuda")
    return torch.as_tensor(CudaArray(ptr, n, typestr), device="cuda")


class EngineBuffers:
    """torch views of a GossipEngine's exchange buffers."""

    def __init__(self, eng: GossipEngine, world=1, buckets=True):
        self.eng = eng
        self.world = world
        self.buckets = buckets
        if buckets:
            sp, rp, bb = eng.bucket_buffers(world)
            self.bucket_words = bb // 4
            self.send = hbm_tensor(sp, world * self.bucket_words, "<i4")
            self.recv = hbm_tensor(rp, world * self.bucket_words, "<i4")
        else:
            ptr, cap = eng.send_buffer()
            self.send = hbm_tensor(ptr, cap)
            self.recv = torch.empty(cap, dtype=torch.int64, device="cuda")

    def rumor_block(self):
        ptr, nbytes = self.eng.rumor_block()
        return hbm_tensor(ptr, nbytes // 8)

    def emit(self):
        self.eng.round_emit_buckets(self.world)

    def merge(self, n_recv=None, run_counts=None):
        if self.buckets:
            self.eng.round_merge_buckets(self.world)
        else:
            self.eng.round_merge_runs(self.recv.data_ptr(), run_counts)

    def ok(self):
        return self.eng.bucket_ok() if self.buckets else self.eng.runs_ok()


def _staged(group, dev):
    # RCCL ("nccl") moves HBM directly; gloo (the CPU rehearsal backend: several ranks
    # sharing one GPU, or CPU stand-ins) needs host tensors, so GPU buffers are staged
    return dist.get_backend(group) == "gloo" and dev.type == "cuda"


def exchange_buckets(recv, send, words, rank, world, stage, group=None):
    """Bucket w of `send` to rank w's slot `rank` of `recv` for every w != rank, one
    grouped batch of sends/receives (the self bucket is read in place by the merge)."""
    if world == 1:
        return
    if stage:
        hs, hr = send.cpu(), torch.empty(recv.shape, dtype=recv.dtype)
    else:
        hs, hr = send, recv
    ops = []
    for w in range(world):
        if w == rank:
            continue
        peer = w if group is None else dist.get_global_rank(group, w)
        ops.append(dist.P2POp(dist.isend, hs[w * words:(w + 1) * words], peer, group))
        ops.append(dist.P2POp(dist.irecv, hr[w * words:(w + 1) * words], peer, group))
    for req in dist.batch_isend_irecv(ops):
        req.wait()
    if stage:
        for w in range(world):
            if w != rank:
                recv[w * words:(w + 1) * words].copy_(hr[w * words:(w + 1) * words])


def all_to_all(out, inp, stage, group=None, out_splits=None, in_splits=None):
    if stage:
        ho = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(ho, inp.cpu(), output_split_sizes=out_splits, input_split_sizes=in_splits,
                               group=group)
        out.copy_(ho)
    else:
        dist.all_to_all_single(out, inp, output_split_sizes=out_splits, input_split_sizes=in_splits, group=group)


class ShardedVivaldi:
    """Vivaldi rounds over members sharded by equal contiguous ranges (one
    CoordinateClients context per rank, created with shard=(lo, hi))."""

    def __init__(self, clients, rank, world, group=None):
        if clients.n % world or clients.hi - clients.lo != clients.n // world:
            raise ValueError("members must be sharded in equal contiguous ranges")
        self.g, self.rank, self.world, self.group = clients, rank, world, group
        b = clients.exchange_buffers(world)
        self.req_send = hbm_tensor(b["req_send"], world * b["req_bucket_bytes"] // 4, "<i4")
        self.req_recv = hbm_tensor(b["req_recv"], world * b["req_bucket_bytes"] // 4, "<i4")
        self.rep_send = hbm_tensor(b["rep_send"], world * b["rep_bucket_bytes"] // 8, "<f8")
        self.rep_recv = hbm_tensor(b["rep_recv"], world * b["rep_bucket_bytes"] // 8, "<f8")
        self.stage = _staged(group, self.req_send.device)
        self._side = None        # the stream the next round's requests go out on
        self._sent = None        # the peer-id pointer whose requests are already out
        self._ev_applied = None  # this round's apply done (it reads the request buckets)
        self._ev_sent = None
        self.time_chunks = False  # round_chunked: time each chunk's observe (chunk_events)
        self.chunk_events = []

    def fetch(self, peer_ptr):
        """Bring the rows of this round's remote peers into the current table."""
        g, w = self.g, self.world
        main = torch.cuda.current_stream()
        if self._sent is not None and self._sent == peer_ptr:
            main.wait_event(self._ev_sent)  # requests built and exchanged during the last observe
        else:
            g.exchange_requests(w, peer_ptr)
            all_to_all(self.req_recv, self.req_send, self.stage, self.group)
        self._sent = None
        g.exchange_serve(w)
        all_to_all(self.rep_recv, self.rep_send, self.stage, self.group)
        g.exchange_apply(w)
        if self._ev_applied is None:
            self._ev_applied = torch.cuda.Event()
        self._ev_applied.record(main)

    def presend(self, next_peer_ptr):
        """The next round's requests, built and exchanged on a side stream while this round's
        observe runs (its peer ids are known ahead: the probe schedule), so the next fetch
        starts at the serve.  Call after this round's fetch, with the context on torch's
        current stream."""
        if self.world == 1 or self._ev_applied is None:
            return
        main = torch.cuda.current_stream()
        if self._side is None:
            self._side = torch.cuda.Stream(device=main.device)
            self._ev_sent = torch.cuda.Event()
        side = self._side
        side.wait_event(self._ev_applied)
        self.g.set_stream(side.cuda_stream)
        try:
            with torch.cuda.stream(side):
                self.g.exchange_requests(self.world, next_peer_ptr)
                all_to_all(self.req_recv, self.req_send, self.stage, self.group)
        finally:
            self.g.set_stream(main.cuda_stream)
        self._ev_sent.record(side)
        self._sent = next_peer_ptr

    def round(self, r, peer_ptr, rtt_ptr, status_ptr=None, slots=16, next_peer_ptr=None, chunks=1):
        if self.world > 1 and chunks > 1:
            return self.round_chunked(r, peer_ptr, rtt_ptr, status_ptr, slots, chunks)
        if self.world > 1:
            self.fetch(peer_ptr)
        self.g.observe(r % slots, peer_ptr, rtt_ptr, status_ptr, r)
        if next_peer_ptr is not None:
            self.presend(next_peer_ptr)

    def round_chunked(self, r, peer_ptr, rtt_ptr, status_ptr=None, slots=16, chunks=4):
        """The round pipelined by member chunks: chunk i is observed while chunk i + 1's remote
        peer rows are requested, served, replied and applied on a side stream, so the exchange
        hides behind the observe instead of preceding it.  Exact: every row served or applied
        is the owner's end-of-previous-round row (coordinate.rs:462-499 reads the peer's last
        coordinate) -- the owners' observe writes the other table, and a remote row applied
        twice (a peer of two chunks) is the same bytes.  Each rank runs the same number of
        chunks, so the all-to-alls pair up across ranks."""
        g, w = self.g, self.world
        main = torch.cuda.current_stream()
        if self._side is None:
            self._side = torch.cuda.Stream(device=main.device)
            self._ev_sent = torch.cuda.Event()
        side = self._side
        n = g.hi - g.lo
        step = -(-n // chunks)
        step = -(-step // 64) * 64  # chunks start at multiples of 64 (one wave's members)
        bounds = [(a, min(n, a + step)) for a in range(0, n, step)]
        bounds += [(n, n)] * (chunks - len(bounds))  # every rank joins every chunk's collectives
        ev_in = torch.cuda.Event()
        ev_in.record(main)  # the previous round's observe (and anything else queued) first
        side.wait_event(ev_in)
        done = []
        g.set_stream(side.cuda_stream)
        try:
            with torch.cuda.stream(side):
                for a, b in bounds:
                    g.exchange_requests(w, peer_ptr, a, b - a)
                    all_to_all(self.req_recv, self.req_send, self.stage, self.group)
                    g.exchange_serve(w)
                    all_to_all(self.rep_recv, self.rep_send, self.stage, self.group)
                    g.exchange_apply(w)
                    ev = torch.cuda.Event()
                    ev.record(side)
                    done.append(ev)
        finally:
            g.set_stream(main.cuda_stream)
        timed = []
        for (a, b), ev in zip(bounds, done):
            main.wait_event(ev)
            if self.time_chunks:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(main)
            g.observe_range(r % slots, peer_ptr, rtt_ptr, a, b - a, status_ptr, r)
            if self.time_chunks:
                e1.record(main)
                timed.append((e0, e1))
        g.flip()
        self.chunk_events.append(timed)
        # the side stream's next use (the next round's requests) must follow this round's observe
        self._ev_applied = torch.cuda.Event()
        self._ev_applied.record(main)
        side.wait_event(self._ev_applied)

    def check(self):
        """True if no request bucket overflowed and every request reached its owner."""
        return self.g.exchange_ok()


class VivaldiTableRefresh:
    """The all-gather variant of the Vivaldi exchange (R = 1 and R = 8):
    after every R-th round each rank's own rows of the table the next round reads are
    all-gathered into every rank's copy, so rows of other shards are up to R rounds old
    (the reference reads a peer's coordinate from its last ack, as stale as the probe
    schedule makes it).  The context's two tables ping-pong every round; with R > 1 an even
    R would always refresh the same one, so the other table's remote rows are brought up to
    date on the device as well."""

    def __init__(self, clients, rank, world, refresh_every=1, group=None):
        if clients.n % world or clients.hi - clients.lo != clients.n // world:
            raise ValueError("members must be sharded in equal contiguous ranges")
        self.g, self.rank, self.world, self.R, self.group = clients, rank, world, int(refresh_every), group
        self.lo, self.hi = clients.lo, clients.hi
        self.stride = clients.table_ptr()[1]
        self.stage = None
        # The gather and the copies below run on torch's current stream: the context's observe
        # kernels must be ordered against it, or the gather could read or overwrite table rows
        # observe is still writing (the context defaults to its own non-blocking stream).  The
        # context is bound to the current stream here; after_round() orders the refresh against
        # the bound stream with stream waits whenever the caller's current stream differs.
        self._bound = None
        if torch.cuda.is_available():
            self._bound = torch.cuda.current_stream().cuda_stream
            clients.set_stream(self._bound)

    def _table(self, ptr):
        t = hbm_tensor(ptr, self.g.n * self.stride, "<f8")
        if self.stage is None:
            self.stage = _staged(self.group, t.device)
        return t

    def after_round(self, r, read_ptr):
        """Call after round r's observe; read_ptr = the table that round read (the
        other one of the pair after the swap)."""
        if self.world == 1 or (r + 1) % self.R:
            return
        ctx = None
        if self._bound is not None and torch.cuda.current_stream().cuda_stream != self._bound:
            # the caller moved to another stream: wait for the context's observe, and make the
            # context's next kernels wait for this refresh
            ctx = torch.cuda.ExternalStream(self._bound)
            torch.cuda.current_stream().wait_stream(ctx)
        self._refresh(read_ptr)
        if ctx is not None:
            ctx.wait_stream(torch.cuda.current_stream())

    def _refresh(self, read_ptr):
        ptr, _ = self.g.table_ptr()
        full = self._table(ptr)
        lo, hi = self.lo * self.stride, self.hi * self.stride
        mine = full[lo:hi].clone()
        if self.stage:  # gloo rehearsal: host-staged
            h = torch.empty(full.shape, dtype=full.dtype)
            dist.all_gather_into_tensor(h, mine.cpu(), group=self.group)
            full.copy_(h)
        else:
            dist.all_gather_into_tensor(full, mine, group=self.group)
        if self.R > 1:
            other = self._table(read_ptr)
            other[:lo].copy_(full[:lo])
            other[hi:].copy_(full[hi:])


class ShardedGossip:
    def __init__(self, cfg: GossipConfig, rank, world, device=0, engine=None, buffers=None, group=None,
                 exchange="buckets"):
        if cfg.n_members % world:
            raise ValueError("n_members must divide evenly over the world")
        per = cfg.n_members // world
        self.rank, self.world, self.group = rank, world, group
        self.shard = (rank * per, (rank + 1) * per)
        if engine is None:
            engine = GossipEngine(dataclasses.replace(cfg, shard=self.shard), device)
            engine.set_stream(torch.cuda.current_stream().cuda_stream)
        self.eng = engine
        want = exchange == "buckets" and world <= MAX_BUCKET_WORLD
        self.buf = buffers if buffers is not None else EngineBuffers(engine, world, want)
        self.buckets = getattr(self.buf, "buckets", False)
        self.dev = self.buf.recv.device
        self.last_in = 0
        self.stage = _staged(group, self.dev)
        self._timing, self._ev = False, []

    def set_timing(self, on):
        """Record stream events around the round's collectives (the rumor-block all-reduce
        and the bucket exchange) for exchange_times(); off by default."""
        self._timing, self._ev = bool(on) and self.dev.type == "cuda", []

    def _mark(self, events, i):
        if self._timing:
            events[i].record()

    def exchange_times(self):
        """Mean ms per timed round of the rumor-block all-reduce and the bucket exchange
        (device time between stream events; synchronises)."""
        if not self._ev:
            return {}
        torch.cuda.synchronize()
        ar = sum(e[0].elapsed_time(e[1]) for e in self._ev) / len(self._ev)
        ex = sum(e[2].elapsed_time(e[3]) for e in self._ev) / len(self._ev)
        return {"rumor_block_all_reduce": ar, "bucket_exchange": ex, "rounds": len(self._ev)}

    def _all_reduce(self, t):
        if self.stage:
            h = t.cpu()
            dist.all_reduce(h, group=self.group)
            t.copy_(h)
        else:
            dist.all_reduce(t, group=self.group)

    def _all_to_all(self, out, inp, out_splits=None, in_splits=None):
        all_to_all(out, inp, self.stage, self.group, out_splits, in_splits)

    def round(self, t, ml=None, acts=None):
        eng, buf = self.eng, self.buf
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if self._timing else None
        eng.round_begin(t, ml, acts)
        blk = buf.rumor_block()
        self._mark(ev, 0)
        if blk.numel():
            self._all_reduce(blk)
        self._mark(ev, 1)
        if self.buckets:
            buf.emit()
            self._mark(ev, 2)
            exchange_buckets(buf.recv, buf.send, buf.bucket_words, self.rank, self.world, self.stage, self.group)
            self._mark(ev, 3)
            buf.merge()
            if ev:
                self._ev.append(ev)
            return None
        counts = eng.round_emit(self.world)
        send_counts = torch.from_numpy(counts.astype(np.int64)).to(self.dev)
        recv_counts = torch.empty_like(send_counts)
        self._all_to_all(recv_counts, send_counts)
        rc = recv_counts.cpu().tolist()
        n_in, n_out = int(sum(rc)), int(counts.sum())
        if n_in > buf.recv.numel():
            raise RuntimeError(f"shard {self.rank}: {n_in} records exceed the receive capacity {buf.recv.numel()}")
        self._all_to_all(buf.recv[:n_in], buf.send[:n_out], rc, [int(x) for x in counts])
        buf.merge(n_in, rc)
        self.last_in = n_in
        return n_out, n_in

    def check(self):
        """True if no exchange capacity was exceeded and every record reached its shard
        (synchronises; call between rounds when validating, and after a timed run)."""
        return self.buf.ok()
