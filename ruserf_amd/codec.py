"""Batched wire codecs over the HIP kernels in csrc/codec.hip.

Mirrors the reference's `Transformable` encode/decode for the hot-path wire
types, in batch:

  * `encode_coordinates` / `decode_coordinates` — Coordinate (core/src/coordinate.rs:663-745),
    optionally behind the PING_VERSION byte of an ack payload (delegate.rs:659-725)
  * `encode_messages` / `decode_messages` — serf frames [tag][Join | Leave | UserEvent]
    (types/src/join.rs, leave.rs, user_event.rs; framing core/src/serf/base.rs:373)

Host numpy in, host numpy out; device memory is torch plumbing.  There is no
CPU path: every call runs the kernels in libruserf_amd.so.
"""
import ctypes as C

import numpy as np

from ._lib import VP, check, lib

SKIPPED = 4
ERR_SHORT, ERR_TYPE, ERR_VARINT, ERR_LEN = -10, -11, -12, -13
PING_VERSION = 1

WIRE_MSG_DTYPE = np.dtype([("type", "u1"), ("flag", "u1"), ("_r0", "<u2"), ("status", "<i4"), ("ltime", "<u8"),
                           ("a_off", "<u8"), ("b_off", "<u8"), ("a_len", "<u4"), ("b_len", "<u4"),
                           ("frame_len", "<u4"), ("_r1", "<u4")])
assert WIRE_MSG_DTYPE.itemsize == 48

_declared = False


def _L():
    global _declared
    L = lib()
    if not _declared:
        i = C.c_int
        for name, args in [
            ("rsf_wire_encoded_lengths", [VP, C.c_uint64, VP, VP]),
            ("rsf_wire_encode", [VP, C.c_uint64, VP, VP, VP, VP, VP]),
            ("rsf_wire_decode", [VP, VP, C.c_uint64, VP, VP]),
            ("rsf_coord_encode", [VP, C.c_uint32, C.c_uint32, C.c_uint64, VP, C.c_uint64, i, VP]),
            ("rsf_coord_decode", [VP, VP, C.c_uint64, i, VP, C.c_uint32, C.c_uint32, VP, VP, VP]),
            ("rsf_vivaldi_ack_payloads", [VP, VP, C.c_uint64, VP, C.c_uint64]),
            ("rsf_vivaldi_observe_acks", [VP, VP, VP, VP, VP, VP, C.c_uint64, C.c_uint32, VP]),
        ]:
            fn = getattr(L, name)
            fn.restype = i
            fn.argtypes = args
        _declared = True
    return L


def _dev(a):
    import torch
    return torch.from_numpy(np.require(a, requirements=["C", "W"])).cuda()


def _empty(n, dtype):
    import torch
    return torch.empty(max(1, n), dtype=dtype, device="cuda")


def _sync():
    import torch
    torch.cuda.synchronize()


def encode_coordinates(rows, dim, ping=False):
    """rows: (n, stride) float64, portion[dim] then error, adjustment, height.
    Returns (bytes uint8 (n, out_stride), out_stride)."""
    import torch
    rows = np.ascontiguousarray(rows, dtype=np.float64)
    n, stride = rows.shape
    out_stride = (1 if ping else 0) + 28 + 8 * dim
    d_rows = _dev(rows)
    d_out = _empty(n * out_stride, torch.uint8)
    check(_L().rsf_coord_encode(d_rows.data_ptr(), dim, stride, n, d_out.data_ptr(), out_stride, int(ping), None))
    _sync()
    return d_out[: n * out_stride].cpu().numpy().reshape(n, out_stride), out_stride


def decode_coordinates(buf, offsets, max_dim=16, ping=False):
    """buf: uint8 bytes; offsets: n+1 uint64.  Returns (rows (n, max_dim+3), dims, status)."""
    import torch
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(off) - 1
    stride = max_dim + 3
    d_buf, d_off = _dev(buf if len(buf) else np.zeros(1, np.uint8)), _dev(off)
    d_rows = _empty(n * stride, torch.float64)
    d_rows.zero_()
    d_dim = _empty(n, torch.int32)
    d_st = _empty(n, torch.int32)
    check(_L().rsf_coord_decode(d_buf.data_ptr(), d_off.data_ptr(), n, int(ping), d_rows.data_ptr(), stride, max_dim,
                                d_dim.data_ptr(), d_st.data_ptr(), None))
    _sync()
    return (d_rows[: n * stride].cpu().numpy().reshape(n, stride), d_dim[:n].cpu().numpy().view(np.uint32),
            d_st[:n].cpu().numpy())


def encode_messages(msgs, blob):
    """msgs: WIRE_MSG_DTYPE records (strings as (offset, length) into blob).
    Returns (frames bytes uint8, offsets n+1 uint64, status int32)."""
    import torch
    msgs = np.ascontiguousarray(msgs, dtype=WIRE_MSG_DTYPE)
    n = len(msgs)
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    d_msgs = _dev(msgs.view(np.uint8) if n else np.zeros(1, np.uint8))
    d_blob = _dev(blob if len(blob) else np.zeros(1, np.uint8))
    d_off = _empty(n + 1, torch.int64)
    L = _L()
    check(L.rsf_wire_encoded_lengths(d_msgs.data_ptr(), n, d_off.data_ptr(), None))
    _sync()
    off = d_off[: n + 1].cpu().numpy().view(np.uint64)
    total = int(off[-1])
    d_out = _empty(total, torch.uint8)
    d_st = _empty(n, torch.int32)
    check(L.rsf_wire_encode(d_msgs.data_ptr(), n, d_blob.data_ptr(), d_off.data_ptr(), d_out.data_ptr(),
                            d_st.data_ptr(), None))
    _sync()
    return d_out[:total].cpu().numpy(), off.copy(), d_st[:n].cpu().numpy()


def decode_messages(buf, offsets):
    """frames [offsets[i], offsets[i+1]) of buf -> WIRE_MSG_DTYPE records (string
    offsets index buf)."""
    import torch
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(off) - 1
    d_buf, d_off = _dev(buf if len(buf) else np.zeros(1, np.uint8)), _dev(off)
    d_out = _empty(n * WIRE_MSG_DTYPE.itemsize, torch.uint8)
    check(_L().rsf_wire_decode(d_buf.data_ptr(), d_off.data_ptr(), n, d_out.data_ptr(), None))
    _sync()
    return d_out[: n * WIRE_MSG_DTYPE.itemsize].cpu().numpy().view(WIRE_MSG_DTYPE).copy()
