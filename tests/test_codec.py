"""Wire codecs: the oracle's restatement pinned by golden bytes
derived from the reference's encode functions, plus round trips and the decode
error paths.  CPU only (the oracle); GPU parity is in test_codec_gpu.py.

Golden bytes: Coordinate per core/src/coordinate.rs:666-692 (u32 BE length,
error, adjustment, height, portion, all f64 big-endian); frames per
core/src/serf/base.rs:373 (tag byte) + types/src/{join,leave,user_event}.rs.
The id / name / payload string encoding (u32 BE length + bytes) and the LEB128
varint come from the un-vendored transformable 0.1: parity unpinned there."""
import ctypes as C
import math

import numpy as np
import pytest

import codec_oracle as CO
import oracle_ffi as O
from ruserf_amd.codec import WIRE_MSG_DTYPE

L = O.lib()


def test_golden_coordinate_bytes():
    # portion [1.0, -2.0, 0.125], error 1.5, adjustment -0.5, height 0.25
    row = np.array([1.0, -2.0, 0.125, 1.5, -0.5, 0.25])
    exp = bytes.fromhex("00000034" "3ff8000000000000" "bfe0000000000000" "3fd0000000000000"
                        "3ff0000000000000" "c000000000000000" "3fc0000000000000")
    assert CO.coord_encode(row, 3).tobytes() == exp
    st, r, d = CO.coord_decode(np.frombuffer(exp, np.uint8))
    assert st == 0 and d == 3 and list(r[:6]) == list(row)


def test_coordinate_round_trip_like_reference():
    """coordinate.rs:860-884: random coordinates survive encode -> decode."""
    rng = np.random.default_rng(0)
    for dim in (1, 3, 8, 16):
        for _ in range(50):
            row = rng.normal(0, 10, dim + 3)
            st, r, d = CO.coord_decode(CO.coord_encode(row, dim))
            assert st == 0 and d == dim
            np.testing.assert_array_equal(r[:dim + 3].view(np.uint64), row.view(np.uint64))
    # non-finite values are carried bit for bit (is_valid is the update's business)
    row = np.array([math.nan, -0.0, math.inf, 1.5, -math.inf, 1e-300])
    st, r, d = CO.coord_decode(CO.coord_encode(row, 3))
    np.testing.assert_array_equal(r[:6].view(np.uint64), row.view(np.uint64))


def test_coordinate_decode_errors():
    good = CO.coord_encode(np.arange(11, dtype=np.float64), 8)
    assert CO.coord_decode(good[:27])[0] == -10          # shorter than the header
    assert CO.coord_decode(good[:-1])[0] == -10          # header length beyond the buffer
    bad = good.copy()
    bad[:4] = [0, 0, 0, 20]                              # below 28: the reference would underflow
    assert CO.coord_decode(bad)[0] == -13
    odd = good.copy()
    odd[:4] = [0, 0, 0, 28 + 8 * 7 + 5]                  # not a multiple of 8: floor (release build)
    st, r, d = CO.coord_decode(odd)
    assert st == 0 and d == 7
    assert CO.coord_decode(good, max_dim=4)[0] == -13    # more dims than the caller's rows hold


def _msg(type_, ltime, a, b=b"", flag=0):
    blob = np.frombuffer(a + b, np.uint8).copy()
    m = np.zeros(1, WIRE_MSG_DTYPE)
    m["type"], m["flag"], m["ltime"] = type_, flag, ltime
    m["a_off"], m["a_len"], m["b_off"], m["b_len"] = 0, len(a), len(a), len(b)
    return m, blob


@pytest.mark.parametrize("case,hexframe", [
    # Join{ltime 300, id "node-1"}: tag 01 | len 16 | varint(300) = ac 02 | u32 6 | "node-1"
    ((1, 300, b"node-1", b"", 0), "01" "00000010" "ac02" "00000006" "6e6f64652d31"),
    # Leave{prune, ltime 5, id "a"}: tag 00 | len 11 | 01 | 05 | u32 1 | "a"
    ((0, 5, b"a", b"", 1), "00" "0000000b" "01" "05" "00000001" "61"),
    # UserEvent{cc, ltime 128, name "deploy", payload 00 ff}: tag 03 | len 23 | 01 | 80 01 | ...
    ((3, 128, b"deploy", b"\x00\xff", 1), "03" "00000017" "01" "8001" "00000006" "6465706c6f79" "00000002" "00ff"),
])
def test_golden_frames(case, hexframe):
    type_, ltime, a, b, flag = case
    m, blob = _msg(type_, ltime, a, b, flag)
    buf, off = CO.wire_encode(m, blob)
    assert buf.tobytes().hex() == hexframe
    d = CO.wire_decode(buf, off)[0]
    assert d["status"] == 0 and d["type"] == type_ and d["ltime"] == ltime and d["flag"] == flag
    assert buf[d["a_off"]:d["a_off"] + d["a_len"]].tobytes() == a
    assert buf[d["b_off"]:d["b_off"] + d["b_len"]].tobytes() == b
    assert d["frame_len"] == len(buf)


def test_varint_edges():
    out = np.zeros(16, np.uint8)
    for v, n in [(0, 1), (127, 1), (128, 2), (16383, 2), (16384, 3), ((1 << 63), 10), ((1 << 64) - 1, 10)]:
        assert L.orc_varint_len(v) == n
        assert L.orc_varint_encode(v, CO.u8p(out)) == n
        got, err = C.c_uint64(), C.c_int(0)
        assert L.orc_varint_decode(CO.u8p(out), n, C.byref(got), C.byref(err)) == n and got.value == v
        assert L.orc_varint_decode(CO.u8p(out), n - 1, C.byref(got), C.byref(err)) == 0 and err.value == -10
    over = np.array([0xFF] * 9 + [0x02], np.uint8)     # 10th byte > 1 overflows u64
    err = C.c_int(0)
    assert L.orc_varint_decode(CO.u8p(over), 10, C.byref(C.c_uint64()), C.byref(err)) == 0 and err.value == -12
    long_ = np.array([0x80] * 11 + [0x00], np.uint8)    # more than 10 bytes
    assert L.orc_varint_decode(CO.u8p(long_), 12, C.byref(C.c_uint64()), C.byref(err)) == 0 and err.value == -12


def test_frame_decode_errors():
    m, blob = _msg(1, 300, b"node-1")
    good, _ = CO.wire_encode(m, blob)
    frames = [b"", bytes([9]) + good[1:].tobytes(), bytes([2]) + good[1:].tobytes(), good[:3].tobytes(),
              good[:-1].tobytes()]
    buf = np.frombuffer(b"".join(frames), np.uint8)
    off = np.cumsum([0] + [len(f) for f in frames]).astype(np.uint64)
    d = CO.wire_decode(buf, off)
    assert list(d["status"]) == [4, -11, -11, -10, -10]
    # Leave's length check is `src.len() + 5 < len` (leave.rs:103): a header 5 bytes
    # past the real length still decodes
    m, blob = _msg(0, 7, b"xy")
    lv, _ = CO.wire_encode(m, blob)
    lv = lv.copy()
    lv[1:5] = np.frombuffer((len(lv) - 1 + 5).to_bytes(4, "big"), np.uint8)
    d = CO.wire_decode(lv, np.array([0, len(lv)], np.uint64))[0]
    assert d["status"] == 0 and d["ltime"] == 7 and d["frame_len"] == len(lv)


def test_random_round_trip_oracle():
    rng = np.random.default_rng(5)
    msgs, blob = CO.random_messages(rng, 2000)
    buf, off = CO.wire_encode(msgs, blob)
    d = CO.wire_decode(buf, off)
    assert np.all(d["status"] == 0)
    for k in ("type", "ltime", "a_len", "b_len"):
        np.testing.assert_array_equal(d[k], msgs[k])
    np.testing.assert_array_equal(d["flag"], np.where(msgs["type"] == 1, 0, msgs["flag"]))  # a Join has no flag
    for i in range(0, 2000, 37):
        a = blob[msgs["a_off"][i]:msgs["a_off"][i] + msgs["a_len"][i]]
        np.testing.assert_array_equal(buf[d["a_off"][i]:d["a_off"][i] + d["a_len"][i]], a)
