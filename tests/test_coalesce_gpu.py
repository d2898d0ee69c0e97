"""UserEventCoalescer on the GPU (many coalescers at once) against the oracle's
restatement (core/src/coalesce/user.rs:52-97, pinned by the reference's
coalescer test in test_oracle_kat.py), applied group by group."""
import ctypes as C

import numpy as np
import pytest

import oracle_ffi as O
from ruserf_amd.coalesce import USER_EVENT_DTYPE, coalesce_user_events

pytestmark = pytest.mark.gpu
L = O.lib()


def oracle_flush(events):
    out = []
    for g in np.unique(events["group"]):
        sel = events[events["group"] == g]
        arr = (O.UEvent * len(sel))()
        for i, e in enumerate(sel):
            arr[i].name, arr[i].ltime, arr[i].payload = int(e["name"]), int(e["ltime"]), int(e["payload"])
        res = (O.UEvent * len(sel))()
        k = L.orc_coalesce_user_events(arr, len(sel), res)
        for i in range(k):
            out.append((int(g), res[i].name, res[i].ltime, res[i].payload))
    return np.array(out, dtype=USER_EVENT_DTYPE) if out else np.zeros(0, USER_EVENT_DTYPE)


@pytest.mark.parametrize("n,groups,names,span", [(20000, 300, 16, 6), (5000, 2, 3, 40), (3000, 3000, 4, 3),
                                                 (1, 1, 1, 1)])
def test_coalesce_matches_oracle(n, groups, names, span):
    rng = np.random.default_rng(n + groups)
    ev = np.zeros(n, USER_EVENT_DTYPE)
    ev["group"] = rng.integers(0, groups, n)
    ev["name"] = rng.integers(0, names, n)
    ev["ltime"] = rng.integers(1, 1 + span, n)
    ev["payload"] = np.arange(n)
    got = coalesce_user_events(ev)
    exp = oracle_flush(ev)
    np.testing.assert_array_equal(got, exp)


def test_coalesce_reference_case():
    """coalesce/user.rs:125-200: foo keeps only ltime 2, bar keeps both ltime-2 events."""
    ev = np.zeros(4, USER_EVENT_DTYPE)
    ev["name"] = [1, 1, 2, 2]        # foo, foo, bar, bar
    ev["ltime"] = [1, 2, 2, 2]
    ev["payload"] = [10, 11, 20, 21]
    got = coalesce_user_events(ev)
    assert list(zip(got["name"], got["ltime"], got["payload"])) == [(1, 2, 11), (2, 2, 20), (2, 2, 21)]
