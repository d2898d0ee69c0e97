"""Gossip round engine: host mirror of ruserf's merge/dissemination surface.

The reference's hot path for membership is driven by memberlist through
`SerfDelegate` (core/src/serf/delegate.rs:111-795): `notify_message`
dispatches to `handle_node_join_intent` / `handle_node_leave_intent` /
`handle_user_event` / `handle_query` (core/src/serf/base.rs), re-queueing the
message when the handler returns true; `broadcast_messages` drains the three
transmit-limited queues; `notify_join` / `notify_leave` call
`handle_node_join` / `handle_node_leave`.  `GossipEngine` holds a whole
cluster (or one shard of it) in HBM and runs those handlers as HIP kernels:

  * `apply_batch(msgs)`   — notify_message over a batch (returns the handler results)
  * `round(t, ml, acts)`  — one full round: memberlist transitions, originations
                            (Serf::join/leave/user_event/query/force_leave), emission
                            (broadcast_messages to k peers), exchange, canonical merge
  * `round_begin/emit/merge` — the same split for multi-GPU sharding (see dist.py)
  * `push_pull(pairs)`    — local_state / merge_remote_state (delegate.rs:376-554) for a
                            batch of (receiver, sender) pairs: push/pull anti-entropy

There is no CPU execution path: every call goes to libruserf_amd.so.
"""
import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._gossip_sigs import RsfGossipCfg
from ._lib import check, lib, ptr

# encodings (include/ruserf_amd.h)
KIND_UNKNOWN, KIND_INTENT_JOIN, KIND_INTENT_LEAVE, KIND_KNOWN = 0, 1, 2, 3
STATUS_NONE, STATUS_ALIVE, STATUS_LEAVING, STATUS_LEFT, STATUS_FAILED = 0, 1, 2, 3, 4
MSG_LEAVE, MSG_JOIN, MSG_USER_EVENT, MSG_QUERY = 0, 1, 3, 4
F_REBROADCAST, F_REFUTE, F_PRUNE, F_DELIVER, F_MEMBER_EVENT = 1, 2, 4, 8, 16
# per-member error bits (members()["err"])
E_EVSLOT, E_QSLOT, E_REFUTE, E_STAGE, E_QUEUE_PRUNE, E_DELIVERY_LOG, E_DEEP_INVARIANT = 1, 2, 4, 8, 16, 32, 64
# QueueOptions defaults (core/src/options.rs:494-530)
MAX_QUEUE_DEPTH, MIN_QUEUE_DEPTH, QUEUE_DEPTH_WARNING = 4096, 0, 128
ACT_JOIN_SELF, ACT_LEAVE_SELF, ACT_FORCE_LEAVE, ACT_USER_EVENT, ACT_QUERY = 1, 2, 3, 4, 5
ML_JOIN, ML_LEAVE, ML_UPDATE = 1, 2, 3
# an origination's result (GossipEngine.action_status): ok, skipped (not this shard's member,
# or its process is down), or the SerfError of the entry point's size checks
# (core/src/error.rs:292-311; api.rs:255-287, base.rs:919-921)
ACT_OK, ACT_SKIPPED = 0, 4
ERR_USER_EVENT_LIMIT, ERR_USER_EVENT_TOO_LARGE, ERR_RAW_USER_EVENT_TOO_LARGE, ERR_QUERY_TOO_LARGE = -20, -21, -22, -23
USER_EVENT_SIZE_LIMIT = 9 * 1024  # core/src/serf.rs:42


def serf_error_text(status, cfg, size=None):
    """The reference's Display text of an origination error (SerfError, error.rs:294-311).
    `size` is the value the reference formats into the message where it is not a limit
    (the encoded length of RawUserEventTooLarge / QueryTooLarge), if the caller has it."""
    if status == ERR_USER_EVENT_LIMIT:
        return f"ruserf: user event exceeds configured limit of {cfg.max_user_event_size} bytes before encoding"
    if status == ERR_USER_EVENT_TOO_LARGE:
        return f"ruserf: user event exceeds sane limit of {USER_EVENT_SIZE_LIMIT} bytes before encoding"
    if status == ERR_RAW_USER_EVENT_TOO_LARGE:
        return f"ruserf: user event exceeds sane limit of {size} bytes after encoding"
    if status == ERR_QUERY_TOO_LARGE:
        return f"ruserf: query exceeds limit of {size} bytes"
    return None
PP_JOIN, PP_EVENT_JOIN_IGNORE = 1, 2

ACTION_DTYPE = np.dtype([("member", "<u4"), ("act", "<u4"), ("subject", "<u4"), ("name_len", "<u4"),
                         ("payload_len", "<u4"), ("flags", "<u4"), ("key", "<u8")])
ML_DTYPE = np.dtype([("subject", "<u4"), ("kind", "<u4"), ("set_alive", "<u4"), ("_r", "<u4")])
MSG_DTYPE = np.dtype([("receiver", "<u4"), ("subject", "<u4"), ("ltime", "<u8"), ("key", "<u8"), ("type", "u1"),
                      ("flags", "u1"), ("_r0", "<u2"), ("_r1", "<u4")])
RUMOR_DTYPE = np.dtype([("ltime", "<u8"), ("key", "<u8"), ("subject", "<u4"), ("type", "u1"), ("flags", "u1"),
                        ("msg_len", "<u2")])
PP_PAIR_DTYPE = np.dtype([("receiver", "<u4"), ("sender", "<u4")])
# kind: DELIVERY_USER_EVENT (ltime, key) or DELIVERY_MEMBER_EVENT (ltime = MemberEventType, key = subject)
DELIVERY_DTYPE = np.dtype([("ltime", "<u8"), ("key", "<u8"), ("member", "<u4"), ("cc", "u1"), ("kind", "u1"),
                           ("_r", "u1", 2)])
DELIVERY_USER_EVENT, DELIVERY_MEMBER_EVENT = 0, 1
assert ACTION_DTYPE.itemsize == 32 and ML_DTYPE.itemsize == 16 and MSG_DTYPE.itemsize == 32
assert RUMOR_DTYPE.itemsize == 24 and DELIVERY_DTYPE.itemsize == 24


@dataclass
class GossipConfig:
    n_members: int
    n_subjects: int
    shard: tuple = None            # (lo, hi); default the whole cluster
    queue_cap: int = 64            # slots per transmit-limited queue
    event_buffer_size: int = 512   # Options::event_buffer_size default
    query_buffer_size: int = 512   # Options::query_buffer_size default
    slot_k: int = 8
    fanout: int = 3                # gossip targets per round
    gossip_limit: int = 8 * 24     # byte budget per gossip message: 8 intents of ~22 B + 2 B overhead
    gossip_overhead: int = 2
    retransmit_mult: int = 4       # memberlist LAN default
    max_refute: int = 4
    max_rumors: int = 1 << 20      # rumor ring (a power of two); ids recycle after a full cycle
    seed: int = 0x5EED5EED
    # deep queues: capacity of the intent / query / event queue (0 = queue_cap); above queue_cap
    # (<= 64) the queue is a register head of queue_cap slots plus an HBM tail (reference
    # max_queue_depth 4096, pruned only by the QueueChecker)
    queue_depth: tuple = None
    # Options::max_user_event_size / query_size_limit (options.rs:519, 526): the origination
    # size checks of Serf::user_event / query_in (api.rs:255-287, base.rs:919-921)
    max_user_event_size: int = 512
    query_size_limit: int = 1024

    def depths(self):
        d = self.queue_depth or (0, 0, 0)
        return [int(x) if x else self.queue_cap for x in d]

    def to_c(self):
        lo, hi = self.shard if self.shard is not None else (0, self.n_members)
        c = RsfGossipCfg(n_members=self.n_members, shard_lo=lo, shard_hi=hi, n_subjects=self.n_subjects,
                         queue_cap=self.queue_cap, event_buffer_size=self.event_buffer_size,
                         query_buffer_size=self.query_buffer_size, slot_k=self.slot_k, fanout=self.fanout,
                         gossip_limit=self.gossip_limit, gossip_overhead=self.gossip_overhead,
                         retransmit_mult=self.retransmit_mult, max_refute=self.max_refute,
                         max_rumors=self.max_rumors, seed=self.seed,
                         max_user_event_size=self.max_user_event_size, query_size_limit=self.query_size_limit)
        c.queue_depth[:] = [int(x) for x in (self.queue_depth or (0, 0, 0))]
        return c


def _p(a):
    return C.c_void_p(a.ctypes.data) if a is not None and len(a) else None


class GossipEngine:
    def __init__(self, cfg: GossipConfig, device=0):
        self.cfg = cfg
        self.device = int(device)
        self.lo, self.hi = cfg.shard if cfg.shard is not None else (0, cfg.n_members)
        self.n_loc = self.hi - self.lo
        h = C.c_void_p()
        c = cfg.to_c()
        check(lib().rsf_gossip_create(C.byref(h), C.byref(c), device))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().rsf_gossip_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- setup
    def set_stream(self, s):
        check(lib().rsf_gossip_set_stream(self._h, C.c_void_p(s)))

    def sync(self):
        check(lib().rsf_gossip_sync(self._h))

    def set_subjects(self, subject_member):
        a = np.ascontiguousarray(subject_member, dtype=np.uint32)
        check(lib().rsf_gossip_set_subjects(self._h, ptr(a, C.c_uint32)))

    def init_views(self, kind, status, ltime):
        k = np.ascontiguousarray(kind, dtype=np.uint8)
        s = np.ascontiguousarray(status, dtype=np.uint8)
        t = np.ascontiguousarray(ltime, dtype=np.uint64)
        check(lib().rsf_gossip_init_views(self._h, ptr(k, C.c_uint8), ptr(s, C.c_uint8), ptr(t, C.c_uint64)))

    def set_view(self, member, subject, kind, status, ltime):
        check(lib().rsf_gossip_set_view(self._h, member, subject, kind, status, ltime))

    def set_alive(self, alive):
        a = np.ascontiguousarray(alive, dtype=np.uint8)
        check(lib().rsf_gossip_set_alive(self._h, ptr(a, C.c_uint8)))

    def set_clocks(self, member, clock, event_clock, query_clock):
        check(lib().rsf_gossip_set_clocks(self._h, member, clock, event_clock, query_clock))

    def set_min_times(self, member, event_min, query_min):
        check(lib().rsf_gossip_set_min_times(self._h, member, event_min, query_min))

    def set_serf_state(self, member, state):
        check(lib().rsf_gossip_set_serf_state(self._h, member, state))

    # ---- SerfDelegate::notify_message over a batch
    def apply_batch(self, msgs):
        msgs = np.ascontiguousarray(msgs, dtype=MSG_DTYPE)
        n = len(msgs)
        flags = np.zeros(n, dtype=np.int32)
        refute = np.zeros(n, dtype=np.uint64)
        check(lib().rsf_gossip_apply_batch(self._h, _p(msgs), n, ptr(flags, C.c_int32), ptr(refute, C.c_uint64)))
        return flags, refute

    # ---- push/pull anti-entropy: merge_remote_state(local_state(sender)) at receiver
    def push_pull(self, pairs, is_join=False, event_join_ignore=False):
        """pairs: (receiver, sender) rows; senders are snapshotted before any merge,
        receivers must be distinct (a symmetric exchange is both directions)."""
        pairs = np.ascontiguousarray(pairs, dtype=PP_PAIR_DTYPE)
        flags = (PP_JOIN if is_join else 0) | (PP_EVENT_JOIN_IGNORE if event_join_ignore else 0)
        check(lib().rsf_gossip_push_pull(self._h, _p(pairs), len(pairs), flags))

    def push_pull_device(self, pairs_ptr, n, is_join=False, event_join_ignore=False):
        """device-pointer variant (asynchronous, unvalidated): the throughput path"""
        flags = (PP_JOIN if is_join else 0) | (PP_EVENT_JOIN_IGNORE if event_join_ignore else 0)
        check(lib().rsf_gossip_push_pull_device(self._h, C.c_void_p(pairs_ptr), n, flags))

    # ---- rounds
    def round(self, t, ml=None, acts=None):
        ml = np.ascontiguousarray(ml if ml is not None else np.zeros(0, ML_DTYPE), dtype=ML_DTYPE)
        acts = np.ascontiguousarray(acts if acts is not None else np.zeros(0, ACTION_DTYPE), dtype=ACTION_DTYPE)
        check(lib().rsf_gossip_round(self._h, t, _p(ml), len(ml), _p(acts), len(acts)))
        self._n_acts = len(acts)

    def action_status(self):
        """Each action of the last round / round_begin: ACT_OK, ACT_SKIPPED, or an ERR_* size
        error (the action then changed nothing).  Synchronises."""
        n = getattr(self, "_n_acts", 0)
        out = np.zeros(n, dtype=np.int32)
        check(lib().rsf_gossip_action_status(self._h, ptr(out, C.c_int32) if n else None, n))
        return out

    def round_begin(self, t, ml=None, acts=None):
        ml = np.ascontiguousarray(ml if ml is not None else np.zeros(0, ML_DTYPE), dtype=ML_DTYPE)
        acts = np.ascontiguousarray(acts if acts is not None else np.zeros(0, ACTION_DTYPE), dtype=ACTION_DTYPE)
        check(lib().rsf_gossip_round_begin(self._h, t, _p(ml), len(ml), _p(acts), len(acts)))
        self._n_acts = len(acts)

    def rumor_block(self):
        p = C.c_void_p()
        b = C.c_uint64()
        check(lib().rsf_gossip_rumor_block(self._h, C.byref(p), C.byref(b)))
        return p.value, b.value

    def round_emit(self, world):
        counts = np.zeros(world, dtype=np.uint64)
        check(lib().rsf_gossip_round_emit(self._h, world, ptr(counts, C.c_uint64)))
        return counts

    def send_buffer(self):
        p = C.c_void_p()
        cap = C.c_uint64()
        check(lib().rsf_gossip_send_buffer(self._h, C.byref(p), C.byref(cap)))
        return p.value, cap.value

    def round_merge(self, recv_ptr, n_recv):
        check(lib().rsf_gossip_round_merge(self._h, C.c_void_p(recv_ptr), n_recv))

    def round_merge_runs(self, recv_ptr, run_counts):
        """Merge the received runs (one per source shard, each receiver-sorted) without a sort."""
        rc = np.ascontiguousarray(run_counts, dtype=np.uint64)
        check(lib().rsf_gossip_round_merge_runs(self._h, C.c_void_p(recv_ptr), ptr(rc, C.c_uint64), len(rc)))

    # ---- the exchange without host synchronisation: fixed-capacity buckets per destination
    def bucket_buffers(self, world):
        """(send ptr, recv ptr, bucket bytes): `world` buckets each, device memory"""
        s, r, b = C.c_void_p(), C.c_void_p(), C.c_uint64()
        check(lib().rsf_gossip_bucket_buffers(self._h, world, C.byref(s), C.byref(r), C.byref(b)))
        return s.value, r.value, b.value

    def round_emit_buckets(self, world):
        check(lib().rsf_gossip_round_emit_buckets(self._h, world))

    def round_merge_buckets(self, world):
        check(lib().rsf_gossip_round_merge_buckets(self._h, world))

    def bucket_ok(self):
        ok = C.c_int()
        check(lib().rsf_gossip_bucket_status(self._h, C.byref(ok)))
        return bool(ok.value)

    def runs_ok(self):
        ok = C.c_int()
        check(lib().rsf_gossip_check_runs(self._h, C.byref(ok)))
        return bool(ok.value)

    # ---- inspection
    def members(self):
        n = self.n_loc
        out = {k: np.zeros(n, dtype=np.uint64) for k in ["clock", "event_clock", "query_clock", "digest"]}
        err = np.zeros(n, dtype=np.uint32)
        ss = np.zeros(n, dtype=np.uint8)
        check(lib().rsf_gossip_dump_members(self._h, ptr(out["clock"], C.c_uint64), ptr(out["event_clock"], C.c_uint64),
                                            ptr(out["query_clock"], C.c_uint64), ptr(out["digest"], C.c_uint64),
                                            ptr(err, C.c_uint32), ptr(ss, C.c_uint8)))
        out["err"] = err
        out["serf_state"] = ss
        return out

    def view(self, with_time=False, rows=None):
        """the view (local rows x subjects, flattened); rows=(row0, count) for a slice"""
        row0, cnt = rows if rows is not None else (0, self.n_loc)
        n = cnt * self.cfg.n_subjects
        lt = np.zeros(n, dtype=np.uint64)
        st = np.zeros(n, dtype=np.uint8)
        kd = np.zeros(n, dtype=np.uint8)
        tm = np.zeros(n, dtype=np.uint32)
        check(lib().rsf_gossip_dump_view_rows(self._h, row0, cnt, ptr(lt, C.c_uint64), ptr(st, C.c_uint8),
                                               ptr(kd, C.c_uint8), ptr(tm, C.c_uint32)))
        return (lt, st, kd, tm) if with_time else (lt, st, kd)

    # ---- Reaper tick (base.rs:519-601): times in rounds
    def reap(self, now, reconnect_timeout, tombstone_timeout, recent_intent_timeout):
        check(lib().rsf_gossip_reap(self._h, now, reconnect_timeout, tombstone_timeout, recent_intent_timeout))

    def set_now(self, now):
        check(lib().rsf_gossip_set_now(self._h, now))

    # ---- delivery log: UserEvents sent to the application (event_tx, base.rs:831-835)
    def set_delivery_log(self, per_member):
        """Log up to per_member deliveries per member per round (0 turns the log off)."""
        self._dcap = int(per_member)
        check(lib().rsf_gossip_set_delivery_log(self._h, self._dcap))

    def deliveries(self):
        """This round's deliveries (DELIVERY_DTYPE), member by member, each in delivery order."""
        cap = self.n_loc * max(1, getattr(self, "_dcap", 0))
        out = np.zeros(cap, dtype=DELIVERY_DTYPE)
        n = C.c_uint64()
        check(lib().rsf_gossip_dump_deliveries(self._h, _p(out), cap, C.byref(n)))
        return out[: n.value]

    # ---- snapshot log + restart (snapshot.rs; base.rs:122-204) and the Reconnector
    def enable_snapshot(self, rejoin_after_leave=False):
        """Start every member's snapshotter (Options::snapshot_path set)."""
        self._snap_w = (self.cfg.n_subjects + 31) // 32
        check(lib().rsf_gossip_enable_snapshot(self._h, int(bool(rejoin_after_leave))))

    def snapshot_files(self, first=None, count=None):
        """The snapshot files of members [first, first+count) (global ids), compacted:
        (offsets u64[count+1], bytes u8) on the host, built on the device."""
        import torch
        first = self.lo if first is None else int(first)
        count = self.n_loc - (first - self.lo) if count is None else int(count)
        dev = torch.device("cuda", self.device)
        offs = torch.empty(count + 1, dtype=torch.int64, device=dev)
        total = C.c_uint64()
        check(lib().rsf_gossip_snapshot_encode(self._h, first, count, C.c_void_p(offs.data_ptr()), None, 0,
                                               C.byref(total)))
        out = torch.empty(max(1, total.value), dtype=torch.uint8, device=dev)
        check(lib().rsf_gossip_snapshot_encode(self._h, first, count, C.c_void_p(offs.data_ptr()),
                                               C.c_void_p(out.data_ptr()), out.numel(), C.byref(total)))
        self.sync()
        return offs.cpu().numpy().view(np.uint64), out[: total.value].cpu().numpy()

    def restart(self, members, files):
        """Restart members (global ids) from snapshot files (bytes each); per member 1 =
        rejoined, 0 = alone, <0 = the file did not replay (member unchanged)."""
        m = np.ascontiguousarray(members, dtype=np.uint32)
        offs = np.zeros(len(m) + 1, dtype=np.uint64)
        offs[1:] = np.cumsum([len(f) for f in files])
        blob = np.frombuffer(b"".join(bytes(f) for f in files) or b"\0", dtype=np.uint8).copy()
        res = np.zeros(len(m), dtype=np.int32)
        check(lib().rsf_gossip_restart(self._h, ptr(m, C.c_uint32), len(m), ptr(blob, C.c_uint8),
                                       ptr(offs, C.c_uint64), res.ctypes.data_as(C.POINTER(C.c_int32))))
        return res

    def snapshot_state(self):
        """(alive bits [n_loc][ceil(S/32)] u32, [n_loc][4] u64 {event clock, query clock,
        clock at leave, flags})"""
        bits = np.zeros((self.n_loc, self._snap_w), dtype=np.uint32)
        st = np.zeros((self.n_loc, 4), dtype=np.uint64)
        check(lib().rsf_gossip_dump_snapshot(self._h, ptr(bits, C.c_uint32), ptr(st, C.c_uint64)))
        return bits, st

    def reconnect(self, tick, target_ptr=None):
        """One Reconnector tick at every member (asynchronous); with target_ptr (device,
        n_loc u32) the tried subject per member (0xFFFFFFFF: none)."""
        check(lib().rsf_gossip_reconnect(self._h, tick, C.c_void_p(target_ptr) if target_ptr else None))

    def reconnect_targets(self, tick):
        """reconnect(tick), returning the targets on the host (synchronises)."""
        import torch
        t = torch.empty(self.n_loc, dtype=torch.int32, device=torch.device("cuda", self.device))
        self.reconnect(tick, t.data_ptr())
        self.sync()
        return t.cpu().numpy().view(np.uint32)

    def pruned(self):
        """Per member: live queue items its bounded queues dropped when full (cumulative)."""
        out = np.zeros(self.n_loc, dtype=np.uint32)
        check(lib().rsf_gossip_dump_pruned(self._h, ptr(out, C.c_uint32), None))
        return out

    def flush(self):
        """Apply every member's pending re-queues to its queues (asynchronous; the
        inspection calls do it themselves)."""
        check(lib().rsf_gossip_flush(self._h))

    def pruned_total(self, flush=True):
        """Sum of pruned() over the shard; flush=False: as of each member's last emission."""
        out = C.c_uint64(0)
        check(lib().rsf_gossip_pruned_total(self._h, 1 if flush else 0, C.byref(out)))
        return int(out.value)

    def expired(self):
        """Per member: queue items dropped at emission because their rumor slot was recycled."""
        out = np.zeros(self.n_loc, dtype=np.uint32)
        check(lib().rsf_gossip_dump_pruned(self._h, None, ptr(out, C.c_uint32)))
        return out

    def check_queues(self, max_queue_depth=MAX_QUEUE_DEPTH, min_queue_depth=MIN_QUEUE_DEPTH,
                     depth_warning=QUEUE_DEPTH_WARNING):
        """One QueueChecker tick (base.rs:703-760) over the intent / query / event queues:
        returns {queued, warn, pruned}, 3 counts each."""
        q, w, p = (np.zeros(3, dtype=np.uint64) for _ in range(3))
        check(lib().rsf_gossip_check_queues(self._h, max_queue_depth, min_queue_depth, depth_warning,
                                            ptr(q, C.c_uint64), ptr(w, C.c_uint64), ptr(p, C.c_uint64)))
        return {"queued": q, "warn": w, "pruned": p}

    def check_queues_phase(self, period, phase, max_queue_depth=MAX_QUEUE_DEPTH, min_queue_depth=MIN_QUEUE_DEPTH,
                           depth_warning=QUEUE_DEPTH_WARNING):
        """A staggered QueueChecker tick: the same tick at the members whose global id is
        phase mod period only (each node's checker runs on its own timer).  Asynchronous;
        the counts accumulate until checker_stats(reset=True)."""
        check(lib().rsf_gossip_check_queues_phase(self._h, max_queue_depth, min_queue_depth, depth_warning,
                                                  int(period), int(phase)))

    def set_checker(self, period, max_queue_depth=MAX_QUEUE_DEPTH, min_queue_depth=MIN_QUEUE_DEPTH,
                    depth_warning=QUEUE_DEPTH_WARNING):
        """In-round staggered QueueChecker ticks: every round r then ticks the members whose
        global id is r mod period, between the round's emission and its merge (period 0:
        off).  Resets the checker counts."""
        check(lib().rsf_gossip_set_checker(self._h, max_queue_depth, min_queue_depth, depth_warning, int(period)))

    def checker_stats(self, reset=False):
        """{queued, warn, pruned} accumulated by the checker ticks since the last reset"""
        q, w, p = (np.zeros(3, dtype=np.uint64) for _ in range(3))
        check(lib().rsf_gossip_checker_stats(self._h, ptr(q, C.c_uint64), ptr(w, C.c_uint64), ptr(p, C.c_uint64),
                                             int(bool(reset))))
        return {"queued": q, "warn": w, "pruned": p}

    def deep_stats(self):
        """(members that took the exact whole-queue emission since creation, since the last call)"""
        a, b = C.c_uint64(), C.c_uint64()
        check(lib().rsf_gossip_deep_stats(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def queues(self, width=None):
        """[n_loc * 3 * D] per field, D = the deepest queue's capacity, each queue in send order;
        width: only each queue's first `width` items (then self.max_live = the most any holds)"""
        w = int(width) if width else max(self.cfg.depths())
        n = self.n_loc * 3 * w
        r = np.zeros(n, dtype=np.uint32)
        sq = np.zeros(n, dtype=np.uint32)
        tx = np.zeros(n, dtype=np.uint16)
        ln = np.zeros(n, dtype=np.uint16)
        ns = np.zeros(self.n_loc * 3, dtype=np.uint32)
        if width:
            ml = C.c_uint32()
            check(lib().rsf_gossip_dump_queues_width(self._h, w, ptr(r, C.c_uint32), ptr(sq, C.c_uint32),
                                                     ptr(tx, C.c_uint16), ptr(ln, C.c_uint16), ptr(ns, C.c_uint32),
                                                     C.byref(ml)))
            self.max_live = ml.value
        else:
            check(lib().rsf_gossip_dump_queues(self._h, ptr(r, C.c_uint32), ptr(sq, C.c_uint32), ptr(tx, C.c_uint16),
                                               ptr(ln, C.c_uint16), ptr(ns, C.c_uint32)))
        return r, sq, tx, ln, ns

    def deep_class_stats(self):
        """members deferred to the whole-queue emission since creation, per LDS capacity
        class: (tiny, small, middle, full depth)"""
        out = np.zeros(4, dtype=np.uint64)
        check(lib().rsf_gossip_deep_class_stats(self._h, ptr(out, C.c_uint64)))
        return out

    def deep_full_items(self):
        """(sum, max) of the items the full-depth deferred class held per member since creation"""
        a, b = C.c_uint64(), C.c_uint64()
        check(lib().rsf_gossip_deep_full_items(self._h, C.byref(a), C.byref(b)))
        return int(a.value), int(b.value)

    def tails(self, q=0):
        """queue q's HBM tail per member as the engine holds it (pending lists not applied):
        (item counts, sealed-prefix lengths), each [n_loc]"""
        cnt = np.zeros(self.n_loc, dtype=np.uint32)
        sealed = np.zeros(self.n_loc, dtype=np.uint32)
        check(lib().rsf_gossip_dump_tails(self._h, q, ptr(cnt, C.c_uint32), ptr(sealed, C.c_uint32)))
        return cnt, sealed

    def checker_occupancy(self):
        """The checker ticks' occupancy since the last reset, before their prunes: {"bin": items per bin,
        "hist": [3, bins] members per bin per queue (the last bin: everything above),
        "max": [3] the most items any member's queue held}"""
        b, nb = C.c_uint32(), C.c_uint32()
        check(lib().rsf_gossip_checker_occupancy(self._h, None, None, C.byref(b), C.byref(nb)))
        h = np.zeros(3 * nb.value, dtype=np.uint32)
        mx = np.zeros(3, dtype=np.uint32)
        check(lib().rsf_gossip_checker_occupancy(self._h, ptr(h, C.c_uint32), ptr(mx, C.c_uint32), None, None))
        return {"bin": b.value, "hist": h.reshape(3, nb.value), "max": mx}

    def queue_lengths(self):
        """[n_loc, 3] items queued per member and queue (intent, query, event), head + tail,
        after applying the pending lists"""
        out = np.zeros(self.n_loc * 3, dtype=np.uint32)
        check(lib().rsf_gossip_queue_lengths(self._h, ptr(out, C.c_uint32)))
        return out.reshape(self.n_loc, 3)

    def queues_rows(self, row0, rows, width):
        """queues of local rows [row0, row0 + rows), each queue's first `width` items in send
        order: (rumor, seq, transmits, len) arrays shaped [rows, 3, width]"""
        n = rows * 3 * width
        r, sq = np.zeros(n, dtype=np.uint32), np.zeros(n, dtype=np.uint32)
        tx, ln = np.zeros(n, dtype=np.uint16), np.zeros(n, dtype=np.uint16)
        ml = C.c_uint32()
        check(lib().rsf_gossip_dump_queues_rows(self._h, row0, rows, width, ptr(r, C.c_uint32), ptr(sq, C.c_uint32),
                                                ptr(tx, C.c_uint16), ptr(ln, C.c_uint16), C.byref(ml)))
        self.max_live = ml.value
        return tuple(a.reshape(rows, 3, width) for a in (r, sq, tx, ln))

    def buffers(self):
        c = self.cfg
        n = self.n_loc
        ebl = np.zeros(n * c.event_buffer_size, dtype=np.uint64)
        ebc = np.zeros(n * c.event_buffer_size, dtype=np.uint32)
        ebk = np.zeros(n * c.event_buffer_size * c.slot_k, dtype=np.uint64)
        qbl = np.zeros(n * c.query_buffer_size, dtype=np.uint64)
        qbc = np.zeros(n * c.query_buffer_size, dtype=np.uint32)
        qbi = np.zeros(n * c.query_buffer_size * c.slot_k, dtype=np.uint32)
        check(lib().rsf_gossip_dump_buffers(self._h, ptr(ebl, C.c_uint64), ptr(ebc, C.c_uint32), ptr(ebk, C.c_uint64),
                                            ptr(qbl, C.c_uint64), ptr(qbc, C.c_uint32), ptr(qbi, C.c_uint32)))
        return ebl, ebc, ebk, qbl, qbc, qbi

    def rumors(self, first, count):
        out = np.zeros(count, dtype=RUMOR_DTYPE)
        check(lib().rsf_gossip_dump_rumors(self._h, first, count, _p(out)))
        return out

    def refutes(self):
        c = self.cfg
        cnt = np.zeros(c.n_subjects, dtype=np.uint32)
        lt = np.zeros(c.n_subjects * c.max_refute, dtype=np.uint64)
        check(lib().rsf_gossip_dump_refutes(self._h, ptr(cnt, C.c_uint32), ptr(lt, C.c_uint64)))
        return cnt, lt

    def last_round_stats(self):
        s = C.c_uint64()
        m = C.c_uint64()
        check(lib().rsf_gossip_last_round_stats(self._h, C.byref(s), C.byref(m)))
        return s.value, m.value

    # ---- measurement
    def set_profiling(self, on=True):
        check(lib().rsf_gossip_set_profiling(self._h, 1 if on else 0))

    def phase_times(self):
        """Summed device ms of [begin, peers + group sort, emit(+exchange), merge] and the rounds covered."""
        ms = (C.c_double * 4)()
        r = C.c_uint32()
        check(lib().rsf_gossip_phase_times(self._h, ms, C.byref(r)))
        return list(ms), r.value

    def cub_canaries(self):
        """[sort, group reduce/scan, run-merge scan]: True if the canary after that hipCUB
        temporary is intact (nothing wrote past the storage the call asked for); synchronises."""
        out = (C.c_int * 3)()
        check(lib().rsf_gossip_debug_canaries(self._h, out))
        return [bool(x) for x in out]

    def merged_total(self):
        t = C.c_uint64()
        check(lib().rsf_gossip_totals(self._h, C.byref(t)))
        return t.value
