"""memberlist SWIM model on the GPU (rsf_swim_*) against the oracle, bit for bit:
entry states, incarnations, state-change ticks, confirmations, own incarnations,
per-message flags and refutation incarnations, over seeded batches and timer ticks.
PARITY UNPINNED against memberlist itself (not vendored in the reference)."""
import numpy as np
import pytest

import oracle_ffi as O
import swim_cases as SC
from ruserf_amd import swim as W

pytestmark = pytest.mark.gpu


def run_pair(n_members, S, lo, hi, seed, rounds=8, batch=3000, k=2):
    subj, st0, inc0 = SC.random_world(n_members, S, seed)
    cfg = W.SwimConfig(n_members=n_members, n_subjects=S, shard=(lo, hi), suspicion_k=k, suspicion_min=20,
                       suspicion_max=90)
    g = W.SwimState(cfg)
    g.set_subjects(subj)
    g.init(st0, inc0, self_incarnation=1)
    o = O.OracleSwim(lo, hi - lo, S, k, g.timeouts, subj, st0, inc0, 1)
    rng = np.random.default_rng(seed)
    left = rng.choice(np.arange(lo, hi), size=max(1, (hi - lo) // 10), replace=False)
    for m in left:
        g.set_left(int(m))
        o.set_left(int(m))
    now = 0
    for r in range(rounds):
        now += 10
        m = SC.random_batch(rng, lo, hi, S, subj, batch, inc_max=4 + r)
        fg, rg = g.apply_batch(m, now)
        fo, ro = o.apply(m, now)
        assert np.array_equal(fg, fo), f"flags differ in round {r}"
        assert np.array_equal(rg, ro), f"refutation incarnations differ in round {r}"
        assert g.tick(now) == o.tick(now)
        dg, do = g.dump(), o.dump()
        for key in do:
            assert np.array_equal(dg[key], do[key]), f"{key} differs after round {r}"
    g.close()
    o.close()


def test_swim_batches_match_oracle():
    run_pair(n_members=300, S=24, lo=0, hi=300, seed=7)


def test_swim_shard_offset_and_no_confirmations():
    run_pair(n_members=1000, S=40, lo=600, hi=1000, seed=11, k=0)


def test_swim_large_batch_dense_collisions():
    # few receivers and subjects, long per-receiver message chains
    run_pair(n_members=64, S=6, lo=0, hi=16, seed=3, rounds=5, batch=20000, k=4)
