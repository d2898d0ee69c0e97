"""UserEventCoalescer (core/src/coalesce/user.rs:52-97) and MemberEventCoalescer
(core/src/coalesce/member.rs:60-118) for many coalescers at once, over the HIP
sort/scan pipelines in csrc/coalesce.hip.  No CPU path."""
import ctypes as C

import numpy as np

from ._lib import VP, check, lib

USER_EVENT_DTYPE = np.dtype([("group", "<u4"), ("name", "<u4"), ("ltime", "<u8"), ("payload", "<u8")])
MEMBER_EVENT_DTYPE = np.dtype([("group", "<u4"), ("node", "<u4"), ("type", "<u4"), ("member", "<u4")])
assert USER_EVENT_DTYPE.itemsize == 24 and MEMBER_EVENT_DTYPE.itemsize == 16
# MemberEventType (core/src/event.rs), as in include/ruserf_amd.h
MEV_JOIN, MEV_LEAVE, MEV_FAILED, MEV_REAP, MEV_UPDATE = 0, 1, 2, 3, 4
NO_EVENT = 0xFF

_declared = False


def _L():
    global _declared
    L = lib()
    if not _declared:
        L.rsf_coalesce_user_events.restype = C.c_int
        L.rsf_coalesce_user_events.argtypes = [VP, C.c_uint64, VP, C.POINTER(C.c_uint64), VP]
        for name, args in [("rsf_member_coalescer_create", [C.POINTER(VP), C.c_uint32, C.c_uint32, C.c_int]),
                           ("rsf_member_coalescer_destroy", [VP]),
                           ("rsf_member_coalescer_flush", [VP, VP, C.c_uint64, VP, C.POINTER(C.c_uint64), VP]),
                           ("rsf_member_coalescer_dump", [VP, VP])]:
            fn = getattr(L, name)
            fn.restype = C.c_int
            fn.argtypes = args
        _declared = True
    return L


def coalesce_user_events_device(in_ptr, n, out_ptr, stream_ptr=None):
    """device pointers; returns the number of flushed events written to out"""
    k = C.c_uint64(0)
    check(_L().rsf_coalesce_user_events(C.c_void_p(in_ptr), n, C.c_void_p(out_ptr), C.byref(k),
                                        C.c_void_p(stream_ptr) if stream_ptr else None))
    return k.value


def coalesce_user_events(events):
    """events: USER_EVENT_DTYPE records in arrival order -> flushed records"""
    import torch
    ev = np.ascontiguousarray(events, dtype=USER_EVENT_DTYPE)
    n = len(ev)
    if n == 0:
        return ev.copy()
    d_in = torch.from_numpy(ev.view(np.uint8).copy()).cuda()
    d_out = torch.empty(n * 24, dtype=torch.uint8, device="cuda")
    k = coalesce_user_events_device(d_in.data_ptr(), n, d_out.data_ptr())
    torch.cuda.synchronize()
    return d_out[: k * 24].cpu().numpy().view(USER_EVENT_DTYPE).copy()


class MemberEventCoalescer:
    """n_groups MemberEventCoalescers (one per event stream, e.g. per member) over n_nodes
    nodes (subject slots), their last_events tables in HBM.  flush(events) = coalesce()
    of one quantum's events in arrival order, then flush(): returns the events sent,
    sorted by (group, type, node)."""

    def __init__(self, n_groups, n_nodes, device=0):
        self.n_groups, self.n_nodes, self.device = int(n_groups), int(n_nodes), int(device)
        self._h = VP()
        check(_L().rsf_member_coalescer_create(C.byref(self._h), self.n_groups, self.n_nodes, self.device))

    def close(self):
        if getattr(self, "_h", None):
            _L().rsf_member_coalescer_destroy(self._h)
            self._h = VP()

    __del__ = close

    def flush_device(self, in_ptr, n, out_ptr, stream_ptr=None):
        k = C.c_uint64(0)
        check(_L().rsf_member_coalescer_flush(self._h, C.c_void_p(in_ptr), n, C.c_void_p(out_ptr), C.byref(k),
                                              C.c_void_p(stream_ptr) if stream_ptr else None))
        return k.value

    def flush(self, events):
        import torch
        ev = np.ascontiguousarray(events, dtype=MEMBER_EVENT_DTYPE)
        n = len(ev)
        if n == 0:
            return ev.copy()
        dev = torch.device("cuda", self.device)
        d_in = torch.from_numpy(ev.view(np.uint8).copy()).to(dev)
        d_out = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        k = self.flush_device(d_in.data_ptr(), n, d_out.data_ptr())
        return d_out[: k * 16].cpu().numpy().view(MEMBER_EVENT_DTYPE).copy()

    def last_events(self):
        out = np.zeros((self.n_groups, self.n_nodes), np.uint8)
        check(_L().rsf_member_coalescer_dump(self._h, C.c_void_p(out.ctypes.data)))
        return out
