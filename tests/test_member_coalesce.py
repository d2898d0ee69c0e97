"""MemberEventCoalescer (core/src/coalesce/member.rs:60-118).

CPU: the oracle restatement against the reference's own tests
(test_member_event_coealesce_basic, test_member_event_coalesce_tag_update, member.rs:152-370).
GPU: the batched coalescer (csrc/coalesce.hip) bit-exact against the oracle over random
streams and several quanta (last_events carried across flushes)."""
import numpy as np
import pytest

import oracle_ffi as O
from ruserf_amd.coalesce import (MEMBER_EVENT_DTYPE, MEV_FAILED, MEV_JOIN, MEV_LEAVE, MEV_REAP, MEV_UPDATE,
                                 NO_EVENT)

FOO, BAR, ZIP, DEAD = 0, 1, 2, 3
TAGS_NONE, TAGS_ROLE_FOO, TAGS_ROLE_BAR = 0, 1, 2


def ev(rows):
    a = np.zeros(len(rows), MEMBER_EVENT_DTYPE)
    for i, (g, node, ty, member) in enumerate(rows):
        a[i] = (g, node, ty, member)
    return a


def by_type(out):
    """the flushed members grouped by type, as the reference's events map"""
    d = {}
    for r in out:
        d.setdefault(int(r["type"]), []).append((int(r["node"]), int(r["member"])))
    return d


def test_member_coalesce_basic_kat():
    """member.rs:152-289: Join foo, Leave foo, Leave bar, Update zip (role=foo), Update zip
    (role=bar), Reap dead -> three events: Leave {bar, foo}, Update {zip with role=bar},
    Reap {dead}; foo's Join is superseded by its Leave."""
    last = np.full((1, 4), NO_EVENT, np.uint8)
    out = O.member_coalesce(last, ev([(0, FOO, MEV_JOIN, TAGS_NONE), (0, FOO, MEV_LEAVE, TAGS_NONE),
                                      (0, BAR, MEV_LEAVE, TAGS_NONE), (0, ZIP, MEV_UPDATE, TAGS_ROLE_FOO),
                                      (0, ZIP, MEV_UPDATE, TAGS_ROLE_BAR), (0, DEAD, MEV_REAP, TAGS_NONE)]))
    got = by_type(out)
    assert len(got) == 3
    assert sorted(n for n, _ in got[MEV_LEAVE]) == [FOO, BAR]
    assert got[MEV_UPDATE] == [(ZIP, TAGS_ROLE_BAR)]
    assert got[MEV_REAP] == [(DEAD, TAGS_NONE)]
    assert list(last[0]) == [MEV_LEAVE, MEV_LEAVE, MEV_UPDATE, MEV_REAP]


def test_member_coalesce_tag_update_kat():
    """member.rs:291-358: an Update is flushed, and a second Update of the same node in a
    later quantum is not suppressed even though the last event was an Update."""
    last = np.full((1, 1), NO_EVENT, np.uint8)
    out1 = O.member_coalesce(last, ev([(0, FOO, MEV_UPDATE, TAGS_ROLE_FOO)]))
    out2 = O.member_coalesce(last, ev([(0, FOO, MEV_UPDATE, TAGS_ROLE_BAR)]))
    assert [(int(r["type"]), int(r["member"])) for r in out1] == [(MEV_UPDATE, TAGS_ROLE_FOO)]
    assert [(int(r["type"]), int(r["member"])) for r in out2] == [(MEV_UPDATE, TAGS_ROLE_BAR)]


def test_member_coalesce_repeat_suppressed_across_quanta():
    """Some(&previous) if previous == ty && ty != Update => skip (member.rs:89-92): a second
    Join of a node already flushed as Join is dropped; a type change goes out."""
    last = np.full((2, 3), NO_EVENT, np.uint8)
    assert len(O.member_coalesce(last, ev([(0, 1, MEV_JOIN, 0), (1, 1, MEV_FAILED, 0)]))) == 2
    assert len(O.member_coalesce(last, ev([(0, 1, MEV_JOIN, 0), (1, 1, MEV_FAILED, 0)]))) == 0
    out = O.member_coalesce(last, ev([(1, 1, MEV_LEAVE, 0), (0, 1, MEV_JOIN, 0), (0, 2, MEV_JOIN, 0)]))
    assert [(int(r["group"]), int(r["node"]), int(r["type"])) for r in out] == [(0, 2, MEV_JOIN), (1, 1, MEV_LEAVE)]


def random_stream(rng, n, groups, nodes):
    a = np.zeros(n, MEMBER_EVENT_DTYPE)
    a["group"] = rng.integers(0, groups, n)
    a["node"] = rng.integers(0, nodes, n)
    a["type"] = rng.choice([MEV_JOIN, MEV_LEAVE, MEV_FAILED, MEV_REAP, MEV_UPDATE], n, p=[.3, .2, .2, .1, .2])
    a["member"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    return a


@pytest.mark.gpu
@pytest.mark.parametrize("groups,nodes,n,quanta", [(1, 4, 50, 6), (300, 40, 20000, 5), (5000, 7, 100000, 3)])
def test_member_coalescer_gpu_matches_oracle(groups, nodes, n, quanta):
    from ruserf_amd.coalesce import MemberEventCoalescer
    rng = np.random.default_rng(groups * 7 + nodes)
    mc = MemberEventCoalescer(groups, nodes)
    last = np.full((groups, nodes), NO_EVENT, np.uint8)
    for q in range(quanta):
        stream = random_stream(rng, n, groups, nodes)
        got = mc.flush(stream)
        exp = O.member_coalesce(last, stream)
        assert np.array_equal(got, exp), q
        assert np.array_equal(mc.last_events(), last), q
    mc.close()


@pytest.mark.gpu
def test_member_coalescer_rejects_out_of_range():
    from ruserf_amd._lib import EngineError
    from ruserf_amd.coalesce import MemberEventCoalescer
    mc = MemberEventCoalescer(4, 4)
    for bad in [(4, 0, MEV_JOIN, 0), (0, 4, MEV_JOIN, 0), (0, 0, 5, 0)]:
        with pytest.raises(EngineError):
            mc.flush(ev([(0, 0, MEV_JOIN, 0), bad]))
    assert np.all(mc.last_events() == NO_EVENT)  # nothing was flushed
    mc.close()
