"""GPU wire codecs against the oracle, byte for byte (encode) and field for field
(decode), on random batches with every varint width and with corrupted frames;
plus the ping seam: ack_payload on the device and notify_ping_complete from the
wire bytes, against the same updates through rsf_vivaldi_update_batch (itself
oracle-checked in test_vivaldi_gpu.py)."""
import numpy as np
import pytest
import torch

import codec_oracle as CO
from ruserf_amd import CoordinateClients, CoordinateOptions
from ruserf_amd import codec as K

pytestmark = pytest.mark.gpu


def test_encode_matches_oracle_bytes():
    rng = np.random.default_rng(11)
    msgs, blob = CO.random_messages(rng, 20000)
    buf, off, st = K.encode_messages(msgs, blob)
    ebuf, eoff = CO.wire_encode(msgs, blob)
    assert np.all(st == 0)
    np.testing.assert_array_equal(off, eoff)
    np.testing.assert_array_equal(buf, ebuf)


def test_decode_matches_oracle_with_corruption():
    rng = np.random.default_rng(12)
    msgs, blob = CO.random_messages(rng, 20000)
    buf, off = CO.wire_encode(msgs, blob)
    frames = [buf[off[i]:off[i + 1]].copy() for i in range(len(msgs))]
    for i in range(0, len(frames), 3):  # every third frame: truncate, retag, or scribble
        f = frames[i]
        k = rng.integers(0, 4)
        if k == 0:
            frames[i] = f[: rng.integers(0, len(f))]
        elif k == 1:
            f[0] = rng.choice([2, 4, 5, 6, 7, 9, 200])
        elif k == 2:
            f[1 + rng.integers(0, 4)] = rng.integers(0, 256)
        else:
            j = rng.integers(1, len(f))
            f[j:] = 0x80  # unterminated varints / lengths
    buf2 = np.concatenate(frames)
    off2 = np.cumsum([0] + [len(f) for f in frames]).astype(np.uint64)
    got = K.decode_messages(buf2, off2)
    exp = CO.wire_decode(buf2, off2)
    np.testing.assert_array_equal(got.view(np.uint8), exp.view(np.uint8))
    assert np.count_nonzero(got["status"] == 0) > len(frames) // 2
    assert set(np.unique(got["status"])) >= {0, -10, -11}


def test_coordinates_match_oracle():
    rng = np.random.default_rng(13)
    for dim in (3, 8, 16):
        rows = rng.normal(0, 1, (3000, dim + 3))
        rows[::97, 0] = np.nan
        rows[::89, -1] = -0.0
        for ping in (False, True):
            b, stride = K.encode_coordinates(rows, dim, ping=ping)
            for i in range(0, 3000, 101):
                exp = CO.coord_encode(rows[i], dim)
                np.testing.assert_array_equal(b[i, 1:] if ping else b[i], exp)
                if ping:
                    assert b[i, 0] == K.PING_VERSION
            off = np.arange(0, 3001, dtype=np.uint64) * np.uint64(stride)
            r, d, st = K.decode_coordinates(b.reshape(-1), off, max_dim=16, ping=ping)
            assert np.all(st == 0) and np.all(d == dim)
            np.testing.assert_array_equal(r[:, :dim + 3].view(np.uint64), rows.view(np.uint64))
    # error paths: empty ping payload, bad version, truncated, short header
    good, stride = K.encode_coordinates(rows[:1], 16, ping=True)
    g = good.reshape(-1)
    cases = [np.zeros(0, np.uint8), np.concatenate([[2], g[1:]]), g[:-1], g[:20]]
    buf = np.concatenate(cases).astype(np.uint8)
    off = np.cumsum([0] + [len(c) for c in cases]).astype(np.uint64)
    _, _, st = K.decode_coordinates(buf, off, ping=True)
    assert list(st) == [K.SKIPPED, K.ERR_TYPE, K.ERR_SHORT, K.ERR_SHORT]


def test_ack_payloads_and_observe_acks_match_update_batch():
    n, slots = 512, 4
    opts = CoordinateOptions()
    a = CoordinateClients(n, slots, opts)
    b = CoordinateClients(n, slots, opts)
    for t in range(6):  # identical non-trivial state (coordinates, filters, windows) in both
        a.round(t)
        b.round(t)
    rng = np.random.default_rng(14)
    stride = 1 + 28 + 8 * 8
    for rnd in range(8):
        members = rng.permutation(n)[:300].astype(np.uint32)
        peers = rng.integers(0, n, 300).astype(np.uint32)
        slot = rng.integers(0, slots, 300).astype(np.uint32)
        rtt = rng.integers(1_000_000, 90_000_000, 300).astype(np.uint64)
        # the peers' ack payloads, encoded on the device from b's table
        d_peers = torch.from_numpy(peers.view(np.int32)).cuda()
        d_pay = torch.empty(300 * stride, dtype=torch.uint8, device="cuda")
        b.ack_payloads_device(d_peers.data_ptr(), 300, d_pay.data_ptr(), stride)
        torch.cuda.synchronize()
        pay = d_pay.cpu().numpy().reshape(300, stride)
        # mangle a few: empty, bad version, truncated, wrong dimensionality
        frames = [pay[i].copy() for i in range(300)]
        frames[0] = np.zeros(0, np.uint8)
        frames[1][0] = 7
        frames[2] = frames[2][:40]
        four, _ = K.encode_coordinates(np.zeros((1, 7)) + 0.5, 4, ping=True)
        frames[3] = four[0]
        buf = np.concatenate(frames)
        off = np.cumsum([0] + [len(f) for f in frames]).astype(np.uint64)
        dev = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()  # noqa: E731
        d_m, d_s, d_b, d_o, d_r = dev(members.view(np.int32)), dev(slot.view(np.int32)), dev(buf), \
            dev(off.view(np.int64)), dev(rtt.view(np.int64))
        d_st = torch.empty(300, dtype=torch.int32, device="cuda")
        b.observe_acks_device(d_m.data_ptr(), d_s.data_ptr(), d_b.data_ptr(), d_o.data_ptr(), d_r.data_ptr(), 300,
                              d_st.data_ptr(), round_=rnd)
        torch.cuda.synchronize()
        st = d_st.cpu().numpy()
        assert list(st[:3]) == [K.SKIPPED, K.ERR_TYPE, K.ERR_SHORT]
        assert st[3] == 1  # DimensionalityMismatch from CoordinateClient::update
        # the same updates through update_batch on context a, with the decoded coordinates
        from ruserf_amd import Coordinate
        keep = np.arange(4, 300)
        rows_b = np.frombuffer(b"".join(p[1:].tobytes() for p in pay[keep]), np.uint8)
        off_k = np.arange(0, len(keep) + 1, dtype=np.uint64) * np.uint64(stride - 1)
        dec, dims, dst = K.decode_coordinates(rows_b, off_k, max_dim=8)
        assert np.all(dst == 0)
        others = [Coordinate.from_row(dec[i], 8) for i in range(len(keep))]
        sa, _ = a.update_batch(members[keep], slot[keep], others, rtt[keep], round_=rnd)
        np.testing.assert_array_equal(st[keep], sa)
        np.testing.assert_array_equal(b.get_rows().view(np.uint64), a.get_rows().view(np.uint64))
    a.close()
    b.close()
