"""Diagnostic: the first round where a queue_cap > 64 run departs from the oracle, with the
departing members' queues (engine and oracle, in send order) before and after that round."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import gossip_harness as H  # noqa: E402
from ruserf_amd import gossip as G  # noqa: E402
from ruserf_amd import workload as W  # noqa: E402

qcap, limit, rate, n = [float(x) if "." in x else int(x) for x in sys.argv[1:5]]
s, rounds = 64, 12
cfg = G.GossipConfig(n_members=n, n_subjects=s, queue_cap=qcap, gossip_limit=limit, gossip_overhead=2,
                     max_rumors=1 << 17, event_buffer_size=64, query_buffer_size=64, slot_k=4)
subj, acts, ml = W.intents_workload(n, s, rounds, rate=rate, seed=qcap + n)
g = G.GossipEngine(cfg)
g.set_subjects(subj)
g.init_views(*W.initial_views(s))
w = H.oracle_world(cfg, subj, W.initial_views(s))


def queue(st, m):
    st = H.normalize_queues(st)
    r = st["q_rumor"].reshape(-1, 3, qcap)[m, 0]
    sq = st["q_seq"].reshape(-1, 3, qcap)[m, 0]
    tx = st["q_tx"].reshape(-1, 3, qcap)[m, 0]
    ln = st["q_len"].reshape(-1, 3, qcap)[m, 0]
    return [(int(a), int(b), int(c), int(d)) for a, b, c, d in zip(r, sq, tx, ln) if a != 0xFFFFFFFF]


prev_e = prev_o = None
for t in range(rounds):
    g.round(t, ml[t], acts[t])
    H.oracle_round(w, t, ml[t], acts[t])
    e, o = H.engine_state(g), H.world_state(w)
    ne, no = H.normalize_queues(e), H.normalize_queues(o)
    bad = [k for k in ne if not np.array_equal(np.asarray(ne[k]), np.asarray(no[k]))]
    if bad:
        print("round", t, "fields", bad)
        rows = set()
        for k in bad:
            x, y = np.asarray(ne[k]), np.asarray(no[k])
            for idx in np.argwhere(x != y)[:20]:
                rows.add(int(idx[0]))
        for m in sorted(rows)[:3]:
            print("member", m, "pending before (engine p_cnt not dumped); queue before round (engine == oracle):")
            print("  ", queue(prev_e, m)[:40])
            print("  engine after :", queue(e, m)[:40])
            print("  oracle after :", queue(o, m)[:40])
            qe, qo = queue(e, m), queue(o, m)
            print("  only engine:", sorted(set(qe) - set(qo)))
            print("  only oracle:", sorted(set(qo) - set(qe)))
        break
    prev_e, prev_o = e, o
else:
    print("all rounds equal")
