"""Vivaldi network coordinates: host mirror of ruserf's coordinate API.

Mirrors core/src/coordinate.rs — `CoordinateOptions` (62-213), `Coordinate`
(508-650), `CoordinateError` (29-40) and `CoordinateClient` (356-500) — over
the HIP engine in libruserf_amd.so.  The reference keeps one
`CoordinateClient` per Serf node (core/src/serf/base.rs:166-173); here a
`CoordinateClients` object holds a whole population in HBM and every update
or estimate runs on the GPU.  There is no CPU compute path.
"""
import ctypes as C
import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from ._lib import (RSF_ERR_DIM_MISMATCH, RSF_ERR_INVALID_COORD, RSF_ERR_INVALID_RTT, RSF_OK,
                   EngineError, RsfCoordOpts, check, lib, ptr)

DEFAULT_SEED = 0x5EED5EED
MAX_RTT_NS = 10 * 1_000_000_000  # coordinate.rs:477


class CoordinateError(Exception):
    """= CoordinateError (coordinate.rs:29-40)."""

    DIMENSIONALITY_MISMATCH = RSF_ERR_DIM_MISMATCH
    INVALID_COORDINATE = RSF_ERR_INVALID_COORD
    INVALID_RTT = RSF_ERR_INVALID_RTT

    def __init__(self, code, rtt_ns=None):
        names = {1: "dimensions aren't compatible", 2: "invalid coordinate",
                 3: f"round trip time not in valid range, duration {rtt_ns}ns is not a value less than 10s"}
        super().__init__(names.get(code, f"error {code}"))
        self.code = code
        self.rtt_ns = rtt_ns


@dataclass
class CoordinateOptions:
    """= CoordinateOptions::new() defaults (coordinate.rs:200-213)."""
    dimensionality: int = 8
    vivaldi_error_max: float = 1.5
    vivaldi_ce: float = 0.25
    vivaldi_cc: float = 0.25
    adjustment_window_size: int = 20
    height_min: float = 10.0e-6
    latency_filter_size: int = 3
    gravity_rho: float = 150.0

    def with_dimensionality(self, d):
        return _replace(self, dimensionality=d)

    def with_height_min(self, h):
        return _replace(self, height_min=h)

    def with_latency_filter_size(self, f):
        return _replace(self, latency_filter_size=f)

    def with_adjustment_window_size(self, w):
        return _replace(self, adjustment_window_size=w)

    def to_c(self):
        o = RsfCoordOpts()
        for k in ["dimensionality", "adjustment_window_size", "latency_filter_size", "vivaldi_error_max",
                  "vivaldi_ce", "vivaldi_cc", "height_min", "gravity_rho"]:
            setattr(o, k, getattr(self, k))
        return o


def _replace(o, **kw):
    d = dict(o.__dict__)
    d.update(kw)
    return CoordinateOptions(**d)


def row_stride(dim):
    return lib().rsf_coord_row_stride(dim)


@dataclass
class Coordinate:
    """= Coordinate (coordinate.rs:508-548); all values in seconds."""
    portion: np.ndarray
    error: float
    adjustment: float
    height: float

    @classmethod
    def with_options(cls, opts: CoordinateOptions):
        # coordinate.rs:568-577
        return cls(np.zeros(opts.dimensionality), opts.vivaldi_error_max, 0.0, opts.height_min)

    @classmethod
    def new(cls):
        return cls.with_options(CoordinateOptions())

    def is_valid(self):
        # coordinate.rs:581-586
        return bool(np.all(np.isfinite(self.portion))) and all(
            math.isfinite(x) for x in (self.error, self.adjustment, self.height))

    def is_compatible_with(self, other):
        return len(self.portion) == len(other.portion)

    def to_row(self, stride=None):
        d = len(self.portion)
        stride = stride or row_stride(d)
        r = np.zeros(stride)
        r[:d] = self.portion
        r[d], r[d + 1], r[d + 2] = self.error, self.adjustment, self.height
        return r

    @classmethod
    def from_row(cls, row, dim):
        return cls(np.array(row[:dim], dtype=np.float64), float(row[dim]), float(row[dim + 1]),
                   float(row[dim + 2]))


class CoordinateClients:
    """A population of CoordinateClients resident in HBM (one per member).

    Methods mirror CoordinateClient: `update` (462-499), `get_coordinate`
    (406-408), `set_coordinate` (412-415), `forget_node` (455-457), `stats`
    (419-423) and `distance_to` (428-430), each batched over members.
    """

    def __init__(self, n_members, peer_slots=16, opts: Optional[CoordinateOptions] = None,
                 seed=DEFAULT_SEED, device=0, shard=None):
        self.opts = opts or CoordinateOptions()
        self.n = int(n_members)
        self.peer_slots = int(peer_slots)
        self.lo, self.hi = shard if shard is not None else (0, self.n)
        self.dim = self.opts.dimensionality
        self.stride = row_stride(self.dim)
        h = C.c_void_p()
        o = self.opts.to_c()
        check(lib().rsf_vivaldi_create(C.byref(h), self.n, self.lo, self.hi, self.peer_slots, C.byref(o),
                                       seed, device))
        self._h = h

    # ---- lifecycle
    def close(self):
        if getattr(self, "_h", None):
            lib().rsf_vivaldi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, hip_stream_ptr):
        check(lib().rsf_vivaldi_set_stream(self._h, C.c_void_p(hip_stream_ptr)))

    def sync(self):
        check(lib().rsf_vivaldi_sync(self._h))

    # ---- CoordinateClient surface
    def get_rows(self, first=0, count=None):
        count = self.n - first if count is None else count
        out = np.empty((count, self.stride), dtype=np.float64)
        check(lib().rsf_vivaldi_get_coordinates(self._h, first, count, ptr(out, C.c_double)))
        return out

    def get_coordinate(self, member) -> Coordinate:
        return Coordinate.from_row(self.get_rows(member, 1)[0], self.dim)

    def set_coordinate(self, member, coord: Coordinate):
        p = np.ascontiguousarray(coord.portion, dtype=np.float64)
        rc = lib().rsf_vivaldi_set_coordinate(self._h, member, ptr(p, C.c_double), len(p), coord.error,
                                              coord.adjustment, coord.height)
        if rc in (RSF_ERR_DIM_MISMATCH, RSF_ERR_INVALID_COORD):
            raise CoordinateError(rc)
        check(rc)

    def forget_node(self, member, peer_slot):
        check(lib().rsf_vivaldi_forget_node(self._h, member, peer_slot))

    def stats(self):
        r = C.c_uint64()
        check(lib().rsf_vivaldi_resets(self._h, C.byref(r)))
        return {"resets": r.value}

    def update_batch(self, members, peer_slots, others: Sequence[Coordinate], rtt_ns, round_=0):
        """Batched update; returns (status codes, updated rows)."""
        n = len(members)
        m = np.ascontiguousarray(members, dtype=np.uint32)
        s = np.ascontiguousarray(peer_slots, dtype=np.uint32)
        rtt = np.ascontiguousarray(rtt_ns, dtype=np.uint64)
        rows = np.zeros((n, self.stride))
        dims = np.empty(n, dtype=np.uint32)
        for i, o in enumerate(others):
            d = len(o.portion)
            dims[i] = d
            if d == self.dim:
                rows[i] = o.to_row(self.stride)
        status = np.empty(n, dtype=np.int32)
        out = np.empty((n, self.stride))
        check(lib().rsf_vivaldi_update_batch(self._h, ptr(m, C.c_uint32), ptr(s, C.c_uint32),
                                             ptr(rows, C.c_double), ptr(dims, C.c_uint32),
                                             ptr(rtt, C.c_uint64), n, round_, ptr(status, C.c_int32),
                                             ptr(out, C.c_double)))
        return status, out

    def update(self, member, peer_slot, other: Coordinate, rtt_ns, round_=0) -> Coordinate:
        """= CoordinateClient::update for one member; raises CoordinateError."""
        st, out = self.update_batch([member], [peer_slot], [other], [rtt_ns], round_)
        if st[0] != RSF_OK:
            raise CoordinateError(int(st[0]), rtt_ns)
        return Coordinate.from_row(out[0], self.dim)

    def distance_to(self, a, b):
        """estimate_rtt batch: Duration nanos from member a[i] to member b[i]."""
        a = np.ascontiguousarray(a, dtype=np.uint32)
        b = np.ascontiguousarray(b, dtype=np.uint32)
        out = np.empty(len(a), dtype=np.uint64)
        check(lib().rsf_vivaldi_estimate_rtt_batch(self._h, ptr(a, C.c_uint32), ptr(b, C.c_uint32), len(a),
                                                   ptr(out, C.c_uint64)))
        return out

    def estimate_rtt_device(self, a_ptr, b_ptr, n, out_ptr):
        check(lib().rsf_vivaldi_estimate_rtt_device(self._h, C.c_void_p(a_ptr), C.c_void_p(b_ptr), n,
                                                    C.c_void_p(out_ptr)))

    # ---- population round (synthetic network)
    def round(self, r):
        """gen_probes(r) into the context's own buffers, then observe (slot r mod peer_slots)."""
        check(lib().rsf_vivaldi_round(self._h, r))

    def gen_probes(self, r, peer_ptr, rtt_ptr):
        """Synthetic probes of round r into device buffers (shard_n u32 peers, shard_n u64 rtt ns)."""
        check(lib().rsf_vivaldi_gen_probes(self._h, r, C.c_void_p(peer_ptr), C.c_void_p(rtt_ptr)))

    def observe(self, slot, peer_ptr, rtt_ptr, status_ptr=None, round_=0):
        """One update per shard member from device-resident probes (see rsf_vivaldi_observe)."""
        check(lib().rsf_vivaldi_observe(self._h, slot, C.c_void_p(peer_ptr), C.c_void_p(rtt_ptr),
                                        C.c_void_p(status_ptr) if status_ptr else None, round_))

    def observe_range(self, slot, peer_ptr, rtt_ptr, first, count, status_ptr=None, round_=0):
        """observe() over shard members [first, first + count) only, without flipping the
        tables (one chunk of a pipelined round; flip() after the last chunk)"""
        check(lib().rsf_vivaldi_observe_range(self._h, slot, C.c_void_p(peer_ptr), C.c_void_p(rtt_ptr),
                                              C.c_void_p(status_ptr) if status_ptr else None, round_, first, count))

    def flip(self):
        check(lib().rsf_vivaldi_flip(self._h))

    # ---- memberlist's probe loop (see ruserf_amd.probe.ProbeLoop)
    def probe(self, r, up_ptr, peer_ptr, rtt_ptr, acked_ptr):
        """Probes of round r with process liveness up[N] (device pointers, asynchronous)."""
        check(lib().rsf_vivaldi_probe(self._h, r, C.c_void_p(up_ptr), C.c_void_p(peer_ptr), C.c_void_p(rtt_ptr),
                                      C.c_void_p(acked_ptr)))

    def probe_acks(self, peer_ptr, acked_ptr, off_ptr, payload_ptr, payload_cap):
        """The acked probes' ack payloads on the wire (device pointers, asynchronous)."""
        check(lib().rsf_vivaldi_probe_acks(self._h, C.c_void_p(peer_ptr), C.c_void_p(acked_ptr),
                                           C.c_void_p(off_ptr), C.c_void_p(payload_ptr), payload_cap))

    # ---- the ping seam from wire bytes (SerfDelegate::ack_payload / notify_ping_complete)
    def ack_payloads_device(self, members_ptr, n, out_ptr, out_stride):
        """[PING_VERSION][Coordinate] of members[i] at out + i*out_stride (device pointers)."""
        from . import codec
        check(codec._L().rsf_vivaldi_ack_payloads(self._h, C.c_void_p(members_ptr), n, C.c_void_p(out_ptr),
                                                   out_stride))

    def observe_acks_device(self, members_ptr, slots_ptr, payload_ptr, off_ptr, rtt_ptr, n, status_ptr, round_=0):
        """notify_ping_complete over n acks (device pointers, asynchronous)."""
        from . import codec
        check(codec._L().rsf_vivaldi_observe_acks(self._h, C.c_void_p(members_ptr), C.c_void_p(slots_ptr),
                                                   C.c_void_p(payload_ptr), C.c_void_p(off_ptr),
                                                   C.c_void_p(rtt_ptr), n, round_, C.c_void_p(status_ptr)))

    def table_ptr(self):
        p = C.c_void_p()
        s = C.c_uint64()
        check(lib().rsf_vivaldi_table(self._h, C.byref(p), C.byref(s)))
        return p.value, s.value

    # ---- targeted peer-row exchange (multi-GPU; see dist.ShardedVivaldi)
    def exchange_buffers(self, world):
        """Device pointers + bucket sizes of the request / reply buckets for `world` shards."""
        from ._lib import RsfVivaldiXbufs
        x = RsfVivaldiXbufs()
        check(lib().rsf_vivaldi_exchange_buffers(self._h, world, C.byref(x)))
        return {k: getattr(x, k) for k, _ in RsfVivaldiXbufs._fields_}

    def exchange_requests(self, world, peer_ptr, first=None, count=None):
        """the round's requests; with first / count those of shard members [first, first + count)"""
        if first is None:
            check(lib().rsf_vivaldi_exchange_requests(self._h, world, C.c_void_p(peer_ptr)))
        else:
            check(lib().rsf_vivaldi_exchange_requests_range(self._h, world, C.c_void_p(peer_ptr), first, count))

    def exchange_serve(self, world):
        check(lib().rsf_vivaldi_exchange_serve(self._h, world))

    def exchange_apply(self, world):
        check(lib().rsf_vivaldi_exchange_apply(self._h, world))

    def exchange_ok(self):
        ok = C.c_int()
        check(lib().rsf_vivaldi_exchange_status(self._h, C.byref(ok)))
        return bool(ok.value)

    def true_rtt_ns(self, a, b):
        o = C.c_uint64()
        check(lib().rsf_vivaldi_true_rtt_ns(self._h, a, b, C.byref(o)))
        return o.value
