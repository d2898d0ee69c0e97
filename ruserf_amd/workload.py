"""Deterministic synthetic workloads for the gossip round (BASELINE.json configs).

These generate the *inputs* of a round — who originates what (Serf::join /
leave / force_leave / user_event / query) and which memberlist transitions
happen — exactly as a real cluster would hand them to Serf.  They are host
numpy, seeded (numpy Philox), identical on every rank, and never compute any
part of the hot path.

  intents_workload : configs[1]/[2] — N members, S tracked subjects, a fraction
                     `rate` of members originates one join/leave intent per round
  churn_workload   : configs[3] — N members, 1% churn (fail or graceful leave via
                     memberlist transitions), plus a user-event + query flood
"""
import numpy as np

from .gossip import (ACT_FORCE_LEAVE, ACT_JOIN_SELF, ACT_LEAVE_SELF, ACT_QUERY, ACT_USER_EVENT, ACTION_DTYPE,
                     KIND_KNOWN, ML_DTYPE, ML_LEAVE, STATUS_ALIVE)


def subjects_for(n, s):
    """Subject slot -> member id, spread evenly over the id space (and over shards)."""
    step = n // s
    return (np.arange(s, dtype=np.uint64) * step).astype(np.uint32)


def initial_views(s, ltime=1):
    """Every member knows every subject as Alive with status_time `ltime`."""
    return (np.full(s, KIND_KNOWN, np.uint8), np.full(s, STATUS_ALIVE, np.uint8), np.full(s, ltime, np.uint64))


def _sample(rng, pool, k):
    k = min(k, len(pool))
    idx = rng.choice(len(pool), size=k, replace=False)
    return pool[np.sort(idx)]


def intents_workload(n, s, rounds, rate=0.01, seed=0x5EED5EED, prune_frac=0.1):
    """Per round: round(rate*n) distinct members originate one intent.  A
    subject member broadcasts its own join (Serf::join -> broadcast_join) or
    leave (Serf::leave); any other member issues force_leave (remove_failed_node,
    base.rs:474-500) about a random subject, a fraction `prune_frac` of them with
    prune (remove_failed_node_prune, api.rs:565 -> handle_prune).  Returns
    (subj_member, [acts per round], [ml per round])."""
    rng = np.random.Generator(np.random.Philox(seed))
    subj_member = subjects_for(n, s)
    member_subj = np.full(n, -1, dtype=np.int64)
    member_subj[subj_member] = np.arange(s)
    k = max(1, int(round(n * rate)))
    acts_all, ml_all = [], []
    for _ in range(rounds):
        orig = np.sort(rng.choice(n, size=k, replace=False)).astype(np.uint32)
        a = np.zeros(k, dtype=ACTION_DTYPE)
        a["member"] = orig
        is_subj = member_subj[orig] >= 0
        coin = rng.integers(0, 2, size=k)
        a["act"] = np.where(is_subj, np.where(coin == 0, ACT_JOIN_SELF, ACT_LEAVE_SELF), ACT_FORCE_LEAVE)
        a["subject"] = np.where(is_subj, 0, rng.integers(0, s, size=k))
        a["flags"] = np.where(is_subj, 0, (rng.random(size=k) < prune_frac).astype(np.uint32))
        acts_all.append(a)
        ml_all.append(np.zeros(0, dtype=ML_DTYPE))
    return subj_member, acts_all, ml_all


def churn_workload(n, rounds, churn=0.01, events_per_round=100, queries_per_round=10, names=16,
                   seed=0x5EED5EED, prune_frac=0.25, oversize=0.0):
    """configs[3]: S = churn*n subjects; each fails (memberlist NotifyLeave ->
    Failed, then a force_leave two rounds later, a fraction `prune_frac` of them
    with prune) or leaves gracefully (Serf::leave, then NotifyLeave three rounds
    later) at a random round; plus per round a user-event flood (16 names, 32-byte
    payloads, cc 50%) and queries.  oversize > 0: that fraction of the events and
    queries get sizes around the default limits (events: name 1..64 + payload 420..560
    bytes against max_user_event_size 512; queries: payload 940..1040 against
    query_size_limit 1024), so some are rejected by the entry points' size checks."""
    rng = np.random.Generator(np.random.Philox(seed))
    s = max(1, int(round(n * churn)))
    subj_member = subjects_for(n, s)
    when = rng.integers(1, max(2, rounds - 4), size=s)
    graceful = rng.integers(0, 2, size=s).astype(bool)
    pruned = rng.random(size=s) < prune_frac
    dead = np.zeros(n, dtype=bool)
    payload_id = 1
    acts_all, ml_all = [], []
    for t in range(rounds):
        ml, fixed = [], []
        for subj in np.nonzero(when == t)[0]:
            if graceful[subj]:
                fixed.append((subj_member[subj], ACT_LEAVE_SELF, 0))
            else:
                ml.append((subj, ML_LEAVE, 0))
        for subj in np.nonzero((when + 3 == t) & graceful)[0]:
            ml.append((subj, ML_LEAVE, 0))
        forced = np.nonzero((when + 2 == t) & ~graceful)[0]
        for subj, _, set_alive in ml:
            dead[subj_member[subj]] = True
        busy = set(int(m) for m, _, _ in fixed)
        live = np.nonzero(~dead)[0].astype(np.uint32)
        live = live[~np.isin(live, np.fromiter(busy, dtype=np.uint32, count=len(busy)))]
        need = events_per_round + queries_per_round + len(forced)
        orig = rng.permutation(_sample(rng, live, need))
        ev, qs, fl = orig[:events_per_round], orig[events_per_round:events_per_round + queries_per_round], \
            orig[events_per_round + queries_per_round:]
        rows = []
        for m, act, subj in fixed:
            rows.append((m, act, subj, 0, 0, 0, 0))
        for m, subj in zip(fl, forced):
            rows.append((m, ACT_FORCE_LEAVE, subj, 0, 0, int(pruned[subj]), 0))
        for m in ev:
            name = int(rng.integers(0, names))
            nl, pl = 8, 32
            if oversize and rng.random() < oversize:
                nl, pl = int(rng.integers(1, 65)), int(rng.integers(420, 561))
            rows.append((m, ACT_USER_EVENT, 0, nl, pl, int(rng.integers(0, 2)), (name << 32) | payload_id))
            payload_id += 1
        for m in qs:
            nl, pl = 8, 16
            if oversize and rng.random() < oversize:
                nl, pl = 8, int(rng.integers(940, 1041))
            rows.append((m, ACT_QUERY, 0, nl, pl, 0, int(rng.integers(0, 1 << 32))))
        a = np.array(rows, dtype=ACTION_DTYPE) if rows else np.zeros(0, ACTION_DTYPE)
        a = a[np.argsort(a["member"], kind="stable")]
        acts_all.append(a)
        mla = np.zeros(len(ml), dtype=ML_DTYPE)
        for i, (subj, kind, set_alive) in enumerate(ml):
            mla[i] = (subj, kind, set_alive, 0)
        ml_all.append(mla)
    return subj_member, acts_all, ml_all
