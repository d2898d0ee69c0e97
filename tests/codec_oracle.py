"""Oracle-side helpers for the wire-codec tests (test infrastructure: the oracle is
only the checker)."""
import ctypes as C

import numpy as np

import oracle_ffi as O
from ruserf_amd.codec import WIRE_MSG_DTYPE

L = O.lib()


def u8p(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def coord_encode(row, dim):
    row = np.ascontiguousarray(row, dtype=np.float64)
    out = np.zeros(28 + 8 * dim, np.uint8)
    n = L.orc_coord_encode(row.ctypes.data_as(C.POINTER(C.c_double)), dim, u8p(out))
    assert n == len(out)
    return out


def coord_decode(b, max_dim=16):
    b = np.ascontiguousarray(b, dtype=np.uint8)
    row = np.zeros(max_dim + 3)
    d = C.c_uint32(0)
    src = u8p(b) if len(b) else u8p(np.zeros(1, np.uint8))
    st = L.orc_coord_decode(src, len(b), max_dim, row.ctypes.data_as(C.POINTER(C.c_double)), C.byref(d))
    return st, row, d.value


def wire_encode(msgs, blob):
    msgs = np.ascontiguousarray(msgs, dtype=WIRE_MSG_DTYPE)
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    bp = u8p(blob) if len(blob) else u8p(np.zeros(1, np.uint8))
    frames, off = [], [0]
    for i in range(len(msgs)):
        m = msgs[i:i + 1]
        n = L.orc_wire_frame_len(m.ctypes.data)
        out = np.zeros(max(1, n), np.uint8)
        w = L.orc_wire_encode(m.ctypes.data, bp, u8p(out))
        assert w == n
        frames.append(out[:n])
        off.append(off[-1] + n)
    buf = np.concatenate(frames) if frames else np.zeros(0, np.uint8)
    return buf, np.array(off, np.uint64)


def wire_decode(buf, off):
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    out = np.zeros(len(off) - 1, WIRE_MSG_DTYPE)
    base = u8p(buf) if len(buf) else u8p(np.zeros(1, np.uint8))
    for i in range(len(off) - 1):
        L.orc_wire_decode(base, int(off[i]), int(off[i + 1] - off[i]), out[i:i + 1].ctypes.data)
    return out


def random_messages(rng, n, max_str=40):
    """n random Join / Leave / UserEvent records over a random blob"""
    from ruserf_amd.gossip import MSG_JOIN, MSG_LEAVE, MSG_USER_EVENT
    blob = rng.integers(0, 256, size=64 * 1024, dtype=np.uint8)
    m = np.zeros(n, WIRE_MSG_DTYPE)
    m["type"] = rng.choice([MSG_JOIN, MSG_LEAVE, MSG_USER_EVENT], size=n)
    m["flag"] = rng.integers(0, 2, size=n)
    # ltimes across every varint width
    bits = rng.integers(0, 65, size=n).astype(np.uint64)
    lt = rng.integers(0, 1 << 62, size=n, dtype=np.uint64) | (rng.integers(0, 4, size=n, dtype=np.uint64) << 62)
    mask = np.where(bits >= 64, np.uint64(0xFFFFFFFFFFFFFFFF),
                    (np.uint64(1) << np.minimum(bits, 63)) - np.uint64(1))
    m["ltime"] = lt & mask
    m["a_len"] = rng.integers(0, max_str, size=n)
    m["b_len"] = np.where(m["type"] == MSG_USER_EVENT, rng.integers(0, max_str, size=n), 0)
    m["a_off"] = rng.integers(0, len(blob) - max_str, size=n)
    m["b_off"] = rng.integers(0, len(blob) - max_str, size=n)
    return m, blob
