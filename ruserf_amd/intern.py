"""Device-side interning of user-event names and payloads (csrc/intern.hip).

A user event's identity `(name, payload)` is compared by value in the reference
(handle_user_event, core/src/serf/base.rs:801-806); the engine carries it as the exact
key (name_id << 32) | payload_id.  `Interner` assigns those ids on the GPU (bytes
compared, ids in first-occurrence order, so they equal a host dict walked in order);
`wire_event_keys` turns decoded wire frames (codec.decode_messages) into keys without
the host.  No CPU path."""
import ctypes as C

import numpy as np

from ._lib import VP, check, lib

NO_STRING = 0xFFFFFFFF

_declared = False


def _L():
    global _declared
    L = lib()
    if not _declared:
        for name, args in [
            ("rsf_interner_create", [C.POINTER(VP), C.c_uint32, C.c_uint64, C.c_int]),
            ("rsf_interner_destroy", [VP]),
            ("rsf_interner_count", [VP, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]),
            ("rsf_intern", [VP, VP, VP, VP, C.c_uint64, VP, VP]),
            ("rsf_wire_event_keys", [VP, VP, VP, VP, C.c_uint64, VP, VP]),
        ]:
            fn = getattr(L, name)
            fn.restype = C.c_int
            fn.argtypes = args
        _declared = True
    return L


class Interner:
    def __init__(self, max_ids=1 << 20, arena_bytes=64 << 20, device=0):
        self._h = VP()
        check(_L().rsf_interner_create(C.byref(self._h), max_ids, arena_bytes, device))

    def close(self):
        if self._h:
            _L().rsf_interner_destroy(self._h)
            self._h = VP()

    __del__ = close

    def count(self):
        n, b = C.c_uint32(), C.c_uint64()
        check(_L().rsf_interner_count(self._h, C.byref(n), C.byref(b)))
        return n.value, b.value

    def intern_device(self, buf_ptr, off_ptr, len_ptr, n, ids_ptr, stream_ptr=None):
        check(_L().rsf_intern(self._h, C.c_void_p(buf_ptr), C.c_void_p(off_ptr), C.c_void_p(len_ptr), n,
                              C.c_void_p(ids_ptr), C.c_void_p(stream_ptr) if stream_ptr else None))

    def intern(self, strings):
        """list of bytes (None: nothing to intern) -> uint32 ids (NO_STRING for None)"""
        import torch
        n = len(strings)
        if n == 0:
            return np.zeros(0, np.uint32)
        lens = np.array([NO_STRING if s is None else len(s) for s in strings], np.uint32)
        sizes = np.where(lens == NO_STRING, 0, lens).astype(np.uint64)
        off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
        blob = b"".join(s for s in strings if s is not None) or b"\0"
        d_buf = torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).cuda()
        d_off = torch.from_numpy(off.view(np.int64)).cuda()
        d_len = torch.from_numpy(lens.view(np.int32)).cuda()
        d_ids = torch.empty(n, dtype=torch.int32, device="cuda")
        self.intern_device(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_ids.data_ptr())
        torch.cuda.synchronize()
        return d_ids.cpu().numpy().view(np.uint32)


def wire_event_keys(names, payloads, buf, msgs):
    """buf: frame bytes (uint8), msgs: codec.WIRE_MSG_DTYPE records decoded from it ->
    uint64 keys ((name_id << 32) | payload_id for user events, 0 otherwise)"""
    import torch
    from .codec import WIRE_MSG_DTYPE
    msgs = np.ascontiguousarray(msgs, dtype=WIRE_MSG_DTYPE)
    n = len(msgs)
    if n == 0:
        return np.zeros(0, np.uint64)
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    d_buf = torch.from_numpy(buf.copy() if len(buf) else np.zeros(1, np.uint8)).cuda()
    d_msgs = torch.from_numpy(msgs.view(np.uint8).copy()).cuda()
    d_keys = torch.empty(n, dtype=torch.int64, device="cuda")
    check(_L().rsf_wire_event_keys(names._h, payloads._h, C.c_void_p(d_buf.data_ptr()),
                                   C.c_void_p(d_msgs.data_ptr()), n, C.c_void_p(d_keys.data_ptr()), None))
    torch.cuda.synchronize()
    return d_keys.cpu().numpy().view(np.uint64)
