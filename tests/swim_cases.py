"""Shared inputs of the SWIM-model tests (memberlist incarnation merge):
seeded message batches over a small shard with heavy (receiver, subject) collisions."""
import numpy as np

from ruserf_amd.swim import MSG_DTYPE, UNKNOWN, suspicion_timeouts  # noqa: F401


def random_world(n_members, S, seed):
    rng = np.random.default_rng(seed)
    subj = rng.choice(n_members, size=S, replace=False).astype(np.uint32)
    state0 = rng.choice([0, 0, 0, 1, 2, 3, UNKNOWN], size=S).astype(np.uint8)
    inc0 = rng.integers(0, 4, size=S).astype(np.uint32)
    return subj, state0, inc0


def random_batch(rng, lo, hi, S, subj, n, inc_max=8):
    m = np.zeros(n, dtype=MSG_DTYPE)
    m["receiver"] = rng.integers(lo, hi, size=n)
    m["subject"] = rng.integers(0, S, size=n)
    m["incarnation"] = rng.integers(0, inc_max, size=n)
    m["type"] = rng.integers(0, 3, size=n)
    # accusers: mostly random members, sometimes the subject itself (a node leaving:
    # dead{from == node}), sometimes the receiver
    frm = rng.integers(0, hi + 8, size=n).astype(np.uint32)
    own = rng.random(n) < 0.15
    frm[own] = subj[m["subject"][own]]
    # some messages about the receiver itself (refutations)
    selfm = rng.random(n) < 0.1
    for i in np.nonzero(selfm)[0]:
        hit = np.nonzero((subj >= lo) & (subj < hi))[0]
        if len(hit):
            s = int(rng.choice(hit))
            m["subject"][i] = s
            m["receiver"][i] = subj[s]
    m["from"] = frm
    return m
