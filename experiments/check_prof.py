"""Diagnostic only: the QueueChecker's deep prune (check_stream_kernel) at the reference's
regime: 1M members, the intent queue 8704 deep, `rounds` rounds with no tick (queues ~24
items a round deep), then one tick over every member timed on the stream; with a library
built with -DRSF_DEEP_PROF=1 (RSF_LIB_PATH) also its shader-clock split per member: pass 1
(keys into LDS), the selects, pass 2 (compaction), the rest.
Usage: check_prof.py [members] [rounds]"""
import ctypes as C
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import bench_gossip as B  # noqa: E402
from ruserf_amd import workload as W  # noqa: E402
from ruserf_amd._lib import lib  # noqa: E402
from ruserf_amd.gossip import GossipEngine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 300
L = lib()
prof = hasattr(L, "rsf_gossip_deep_prof")
if prof:
    L.rsf_gossip_deep_prof.restype = C.c_int
    L.rsf_gossip_deep_prof.argtypes = [C.POINTER(C.c_uint64)]
cfg = B.gossip_cfg(n, rounds, 1, queue_depth=8704, ring_rounds=rounds)
subj, acts, ml = W.intents_workload(n, B.SUBJECTS, rounds, rate=0.01, seed=B.SEED, prune_frac=B.PRUNE_FRAC)
torch.cuda.set_stream(torch.cuda.Stream())
eng = GossipEngine(cfg)
eng.set_stream(torch.cuda.current_stream().cuda_stream)
eng.set_subjects(subj)
eng.init_views(*W.initial_views(B.SUBJECTS))
for t in range(rounds):
    eng.round(t, ml[t], acts[t])
eng.flush()
torch.cuda.synchronize()
buf = (C.c_uint64 * 80)()
have = prof and L.rsf_gossip_deep_prof(buf) == 0
t0 = time.perf_counter()
st = eng.check_queues(4096, 0, 128)
ms = (time.perf_counter() - t0) * 1e3
out = {"members": n, "rounds": rounds, "tick_ms": round(ms, 2), "queued": int(st["queued"][0]),
       "pruned": int(st["pruned"][0])}
if have:
    L.rsf_gossip_deep_prof(buf)
    v = [int(x) for x in buf]
    m = max(1, v[69])
    out["prof"] = {"members": v[69], "items_per_member": v[68] / m,
                   "cycles_per_member": {"pass1": v[64] / m, "selects": v[65] / m, "pass2": v[66] / m,
                                         "rest": v[67] / m}}
print(json.dumps(out), flush=True)
eng.close()
