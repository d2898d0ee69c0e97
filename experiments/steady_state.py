"""Diagnostic: the bench workload's intent queues over a long run at the reference's queue
semantics -- QueueChecker ticks every K rounds (max_queue_depth 4096), a rumor ring sized
so nothing expires, and a queue depth (register head + HBM tail) as deep as the build allows.
Every `every` rounds it prints one JSON line: ms per round over the window, intent-queue
occupancy (mean / p50 / p99 / max over members), deferred members per round per LDS class,
bounded-queue drops (between ticks; the reference drops none) and ring expiries.
With mode "stagger" each member ticks on its own phase (member id mod check_every) after every
round instead (rsf_gossip_check_queues_phase), inside the timed windows.
Mode "inround": the same staggered ticks inside the rounds (rsf_gossip_set_checker).
Usage: steady_state.py [members] [rounds] [check_every] [depth] [every] [sync|stagger|inround]"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import bench_gossip as B  # noqa: E402
from ruserf_amd import workload as W  # noqa: E402
from ruserf_amd.gossip import GossipEngine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 450
check_every = int(sys.argv[3]) if len(sys.argv) > 3 else 150
depth = int(sys.argv[4]) if len(sys.argv) > 4 else 4096
every = int(sys.argv[5]) if len(sys.argv) > 5 else 10
stagger = len(sys.argv) > 6 and sys.argv[6] == "stagger"
inround = len(sys.argv) > 6 and sys.argv[6] == "inround"
cfg = B.gossip_cfg(n, rounds, 1, queue_depth=depth, ring_rounds=rounds)
print(json.dumps({"members": n, "rounds": rounds, "check_every": check_every, "depth": cfg.depths()[0],
                  "max_rumors": cfg.max_rumors, "stagger": stagger, "inround": inround}), flush=True)
subj, acts, ml = W.intents_workload(n, B.SUBJECTS, rounds, rate=0.01, seed=B.SEED, prune_frac=B.PRUNE_FRAC)
torch.cuda.set_stream(torch.cuda.Stream())
eng = GossipEngine(cfg)
eng.set_stream(torch.cuda.current_stream().cuda_stream)
eng.set_subjects(subj)
eng.init_views(*W.initial_views(B.SUBJECTS))
if inround:
    eng.set_checker(check_every, 4096, 0, 128)
cls0 = eng.deep_class_stats()
pr0, ex0 = 0, 0
t0 = time.perf_counter()
for t in range(rounds):
    eng.round(t, ml[t], acts[t])
    if stagger:
        eng.check_queues_phase(check_every, (t + 1) % check_every, 4096, 0, 128)
    tick = not (stagger or inround) and check_every and (t + 1) % check_every == 0
    if (t + 1) % every == 0 or tick:
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / every * 1e3
        ql = eng.queue_lengths()[:, 0]
        cls = eng.deep_class_stats()
        pr = int(eng.pruned().sum())
        ex = int(eng.expired().sum())
        rec = {"round": t + 1, "ms_per_round": round(ms, 3),
               "occ": {"mean": float(ql.mean()), "p50": int(np.percentile(ql, 50)),
                       "p99": int(np.percentile(ql, 99)), "max": int(ql.max())},
               "deferred_per_round": [(int(a) - int(b)) / every for a, b in zip(cls, cls0)],
               "bounded_pruned": pr - pr0, "expired": ex - ex0}
        if stagger or inround:
            cs = eng.checker_stats(reset=True)
            rec["ticks"] = {"pruned_per_round": int(cs["pruned"][0]) / every}
        if tick:
            torch.cuda.synchronize()
            tt = time.perf_counter()
            st = eng.check_queues(4096, 0, 128)
            tick_ms = (time.perf_counter() - tt) * 1e3
            rec["tick"] = {"queued": int(st["queued"][0]), "pruned": int(st["pruned"][0]),
                           "warn_members": int(st["warn"][0]), "ms": round(tick_ms, 2)}
        print(json.dumps(rec), flush=True)
        cls0, pr0, ex0 = cls, pr, ex
        torch.cuda.synchronize()
        t0 = time.perf_counter()
eng.close()
