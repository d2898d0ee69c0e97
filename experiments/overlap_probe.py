"""Diagnostic: how much would co-scheduling two latency-bound phases gain?  Two independent
gossip contexts (n members each, the bench workload) on two HIP streams: their rounds run
back to back on one stream, then concurrently on two (the launches interleave, so one
context's emission can overlap the other's merge).  If the concurrent pair costs much less
than twice a single round, overlapping emit and merge of one round pipeline would pay.
Usage: overlap_probe.py [members] [rounds]"""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import bench_gossip as B  # noqa: E402
from ruserf_amd import workload as W  # noqa: E402
from ruserf_amd.gossip import GossipEngine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
settle = 17
rounds = settle + 3 * steps
cfg = B.gossip_cfg(n, rounds, 1)
subj, acts, ml = W.intents_workload(n, B.SUBJECTS, rounds, rate=0.01, seed=B.SEED, prune_frac=B.PRUNE_FRAC)
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
engs = []
for k in range(2):
    e = GossipEngine(cfg)
    e.set_stream(streams[k].cuda_stream)
    e.set_subjects(subj)
    e.init_views(*W.initial_views(B.SUBJECTS))
    engs.append(e)
t = 0
for _ in range(settle):
    for e in engs:
        e.round(t, ml[t], acts[t])
    t += 1
torch.cuda.synchronize()


def timed(fn, k):
    global t
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn(t)
        t += 1
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


one = timed(lambda r: engs[0].round(r, ml[r], acts[r]), steps)
pair_serial = timed(lambda r: [engs[0].round(r, ml[r], acts[r]), torch.cuda.synchronize(),
                               engs[1].round(r, ml[r], acts[r]), torch.cuda.synchronize()], steps)
pair_conc = timed(lambda r: [e.round(r, ml[r], acts[r]) for e in engs], steps)
print(json.dumps({"members_each": n, "one_round_ms": one, "pair_serial_ms": pair_serial,
                  "pair_concurrent_ms": pair_conc, "concurrent_over_serial": pair_conc / pair_serial}))
for e in engs:
    e.close()
