"""UserEventCoalescer (core/src/coalesce/user.rs:52-97) for many coalescers at
once, over the HIP sort/scan pipeline in csrc/coalesce.hip.  No CPU path."""
import ctypes as C

import numpy as np

from ._lib import VP, check, lib

USER_EVENT_DTYPE = np.dtype([("group", "<u4"), ("name", "<u4"), ("ltime", "<u8"), ("payload", "<u8")])
assert USER_EVENT_DTYPE.itemsize == 24

_declared = False


def _L():
    global _declared
    L = lib()
    if not _declared:
        L.rsf_coalesce_user_events.restype = C.c_int
        L.rsf_coalesce_user_events.argtypes = [VP, C.c_uint64, VP, C.POINTER(C.c_uint64), VP]
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
