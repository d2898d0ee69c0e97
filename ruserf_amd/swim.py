"""memberlist SWIM layer model on the GPU.

`SwimState` holds, for every member of a shard, memberlist's `nodeMap` entries of the
S tracked subjects -- state, incarnation, state-change tick and the running suspicion
timer -- plus the member's own incarnation.  `apply_batch` is `aliveNode` /
`suspectNode` / `deadNode` for a batch of received messages (one receiver's messages in
array order), `tick` fires the due suspicion timers (`deadNode` from the receiver).

memberlist-core 0.2 is not vendored in the reference (reference Cargo.toml:27-29;
serf reaches it from core/src/serf/base.rs:208-225 and the delegate hooks of
core/src/serf/delegate.rs), so this row's parity is UNPINNED: the kernels
(ruserf_amd/csrc/swim.hip) and the oracle (oracle/oracle.c, orc_swim_*) restate
memberlist's published state machine identically, and the tests compare the two.
"""
import ctypes as C
import math
from dataclasses import dataclass

import numpy as np

from ._lib import P8, P32, PI32, VP, check, lib, ptr

ALIVE, SUSPECT, DEAD, LEFT, UNKNOWN = 0, 1, 2, 3, 255
MSG_ALIVE, MSG_SUSPECT, MSG_DEAD = 0, 1, 2
F_REBROADCAST, F_REFUTE, F_NOTIFY_JOIN, F_NOTIFY_LEAVE, F_SUSPECT, F_CONFIRM = 1, 2, 4, 8, 16, 32
MAX_CONFIRM = 4

MSG_DTYPE = np.dtype([("receiver", "<u4"), ("subject", "<u4"), ("incarnation", "<u4"), ("from", "<u4"),
                      ("type", "<u4"), ("_reserved", "<u4")])


class RsfSwimCfg(C.Structure):
    _fields_ = [("n_members", C.c_uint64), ("shard_lo", C.c_uint64), ("shard_hi", C.c_uint64),
                ("n_subjects", C.c_uint32), ("suspicion_k", C.c_uint32),
                ("timeout", C.c_uint32 * (MAX_CONFIRM + 1)), ("_reserved", C.c_uint32)]


def suspicion_timeouts(k, min_ticks, max_ticks):
    """memberlist's suspicion timeout after c = 0..k confirmations:
    max - log(c+1)/log(k+1) * (max - min), floored, at least min; k < 1 -> min."""
    out = [0] * (MAX_CONFIRM + 1)
    for c in range(MAX_CONFIRM + 1):
        if k < 1:
            out[c] = min_ticks
            continue
        cc = min(c, k)
        frac = math.log(cc + 1.0) / math.log(k + 1.0)
        raw = float(max_ticks) - frac * float(max_ticks - min_ticks)
        out[c] = max(min_ticks, int(math.floor(raw)))
    return out


def _declare(L):
    if getattr(L, "_swim_declared", False):
        return
    i = C.c_int

    def sig(name, args):
        fn = getattr(L, name)
        fn.restype = i
        fn.argtypes = args

    sig("rsf_swim_create", [C.POINTER(VP), C.POINTER(RsfSwimCfg), i])
    sig("rsf_swim_destroy", [VP])
    sig("rsf_swim_set_stream", [VP, VP])
    sig("rsf_swim_set_subjects", [VP, P32])
    sig("rsf_swim_init", [VP, P8, P32, C.c_uint32])
    sig("rsf_swim_set_left", [VP, C.c_uint64, C.c_uint8])
    sig("rsf_swim_apply_batch", [VP, VP, C.c_uint64, C.c_uint32, PI32, P32])
    sig("rsf_swim_tick", [VP, C.c_uint32, C.POINTER(C.c_uint64)])
    sig("rsf_swim_dump", [VP, C.c_uint64, C.c_uint64, P8, P32, P32, P8, P32])
    sig("rsf_swim_probe_failures", [VP, VP, VP, VP, C.c_uint32, VP])
    L._swim_declared = True


@dataclass
class SwimConfig:
    n_members: int
    n_subjects: int
    shard: tuple = None
    suspicion_k: int = 2               # SuspicionMult (4) - 2
    suspicion_min: int = 5000          # ticks (ms): SuspicionMult * log10(n) * ProbeInterval in memberlist
    suspicion_max: int = 30000         # SuspicionMaxTimeoutMult * min


class SwimState:
    def __init__(self, cfg: SwimConfig, device=0):
        L = lib()
        _declare(L)
        lo, hi = cfg.shard or (0, cfg.n_members)
        self.cfg, self.lo, self.hi = cfg, lo, hi
        c = RsfSwimCfg(n_members=cfg.n_members, shard_lo=lo, shard_hi=hi, n_subjects=cfg.n_subjects,
                       suspicion_k=cfg.suspicion_k)
        for j, t in enumerate(suspicion_timeouts(cfg.suspicion_k, cfg.suspicion_min, cfg.suspicion_max)):
            c.timeout[j] = t
        self.timeouts = list(c.timeout)
        self._h = VP()
        check(L.rsf_swim_create(C.byref(self._h), C.byref(c), device))

    def close(self):
        if self._h:
            lib().rsf_swim_destroy(self._h)
            self._h = VP()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_subjects(self, subject_member):
        a = np.ascontiguousarray(subject_member, dtype=np.uint32)
        check(lib().rsf_swim_set_subjects(self._h, ptr(a, C.c_uint32)))

    def init(self, state, incarnation, self_incarnation=1):
        s = np.ascontiguousarray(state, dtype=np.uint8)
        i = np.ascontiguousarray(incarnation, dtype=np.uint32)
        check(lib().rsf_swim_init(self._h, ptr(s, C.c_uint8), ptr(i, C.c_uint32), self_incarnation))

    def set_stream(self, hip_stream_ptr):
        check(lib().rsf_swim_set_stream(self._h, C.c_void_p(hip_stream_ptr)))

    def probe_failures(self, target_ptr, acked_ptr, up_ptr, now, flags_ptr=None):
        """probeNode's failure path at every receiver of the shard (device pointers, see
        rsf_swim_probe_failures): a probe without ack suspects its (tracked) target."""
        check(lib().rsf_swim_probe_failures(self._h, C.c_void_p(target_ptr), C.c_void_p(acked_ptr),
                                            C.c_void_p(up_ptr) if up_ptr else None, now,
                                            C.c_void_p(flags_ptr) if flags_ptr else None))

    def set_left(self, member, left=True):
        check(lib().rsf_swim_set_left(self._h, member, 1 if left else 0))

    def apply_batch(self, msgs, now):
        """aliveNode / suspectNode / deadNode of each message (structured array of MSG_DTYPE);
        returns (flags, refute incarnations)."""
        m = np.ascontiguousarray(msgs, dtype=MSG_DTYPE)
        n = len(m)
        flags = np.zeros(n, dtype=np.int32)
        ref = np.zeros(n, dtype=np.uint32)
        if n:
            check(lib().rsf_swim_apply_batch(self._h, m.ctypes.data, n, now, ptr(flags, C.c_int32),
                                             ptr(ref, C.c_uint32)))
        return flags, ref

    def tick(self, now):
        f = C.c_uint64()
        check(lib().rsf_swim_tick(self._h, now, C.byref(f)))
        return int(f.value)

    def dump(self, first=0, count=None):
        count = (self.hi - self.lo - first) if count is None else count
        S = self.cfg.n_subjects
        st = np.zeros(count * S, np.uint8)
        inc = np.zeros(count * S, np.uint32)
        ch = np.zeros(count * S, np.uint32)
        nc = np.zeros(count * S, np.uint8)
        si = np.zeros(count, np.uint32)
        check(lib().rsf_swim_dump(self._h, first, count, ptr(st, C.c_uint8), ptr(inc, C.c_uint32),
                                  ptr(ch, C.c_uint32), ptr(nc, C.c_uint8), ptr(si, C.c_uint32)))
        return {"state": st.reshape(count, S), "incarnation": inc.reshape(count, S),
                "change": ch.reshape(count, S), "n_confirm": nc.reshape(count, S), "self_incarnation": si}
