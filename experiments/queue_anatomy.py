"""Diagnostic: what a deep intent queue holds at the bench workload (1M members, depth 4096 +
head, ring sized so nothing expires), after R rounds: per (transmits, length) class counts over
a sample of members, the rank in send order where each class starts, and seq ages.
Usage: queue_anatomy.py [members] [rounds] [sample]"""
import collections
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench_gossip as B  # noqa: E402
from ruserf_amd import workload as W  # noqa: E402
from ruserf_amd.gossip import GossipEngine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 110
sample = int(sys.argv[3]) if len(sys.argv) > 3 else 64
cfg = B.gossip_cfg(n, rounds, 1, queue_depth=4096, ring_rounds=rounds)
subj, acts, ml = W.intents_workload(n, B.SUBJECTS, rounds, rate=0.01, seed=B.SEED, prune_frac=B.PRUNE_FRAC)
eng = GossipEngine(cfg)
eng.set_subjects(subj)
eng.init_views(*W.initial_views(B.SUBJECTS))
for t in range(rounds):
    eng.round(t, ml[t], acts[t])
torch.cuda.synchronize()
W_ = cfg.depths()[0]
rows = np.linspace(0, n - 1, sample).astype(np.int64)
cls = collections.Counter()
first_rank = collections.defaultdict(list)
sizes, tx0s, heads_tx0 = [], [], []
for r in rows:
    rid, seq, tx, ln = eng.queues_rows(int(r), 1, W_)
    live = rid[0, 0] != 0xFFFFFFFF
    k = int(live.sum())
    sizes.append(k)
    t, L, sq = tx[0, 0, :k], ln[0, 0, :k], seq[0, 0, :k]
    tx0s.append(int((t == 0).sum()))
    heads_tx0.append(int((t[:64] == 0).sum()))
    seen = set()
    for i in range(k):
        key = (int(t[i]), int(L[i]))
        cls[key] += 1
        if key not in seen:
            seen.add(key)
            first_rank[key].append(i)
out = {"members": n, "rounds": rounds, "sample": sample, "queue_items_mean": float(np.mean(sizes)),
       "tx0_items_mean": float(np.mean(tx0s)), "tx0_items_max": int(np.max(tx0s)),
       "tx0_in_first64_mean": float(np.mean(heads_tx0)),
       "classes_per_member": {f"tx{a}_len{b}": round(v / sample, 2) for (a, b), v in sorted(cls.items())},
       "class_first_rank_median": {f"tx{a}_len{b}": int(np.median(v)) for (a, b), v in sorted(first_rank.items())}}
print(json.dumps(out))
eng.close()
