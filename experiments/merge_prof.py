"""Diagnostic only: per-phase shader-clock totals of merge_kernel (or, with argv[2] ==
"emit" and a -DRSF_EMIT_PROF=1 library, of emit_kernel) at the bench's
1M-member gossip workload (needs a library built with -DRSF_MERGE_PROF=1, loaded
via RSF_LIB_PATH).  Phases: 0 setup (segment bounds, queue + register loads),
1 chunk loads (records, rumors, view entries, chains, clock scan), 2 chain walk,
3 serial part (digest, refutes, re-queue inserts), 4 stores; 5 total; 6 waves."""
import ctypes as C
import json
import sys

import torch

sys.path.insert(0, ".")
import bench_gossip as B  # noqa: E402
from ruserf_amd import workload as W  # noqa: E402
from ruserf_amd._lib import lib  # noqa: E402
from ruserf_amd.gossip import GossipEngine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
L = lib()
L.rsf_gossip_merge_prof.restype = C.c_int
L.rsf_gossip_merge_prof.argtypes = [C.POINTER(C.c_uint64)]
rounds = B.SETTLE_ROUNDS + 5
cfg = B.gossip_cfg(n, rounds, 1)
subj, acts, ml = W.intents_workload(n, B.SUBJECTS, rounds, rate=0.01, seed=B.SEED)
eng = GossipEngine(cfg)
eng.set_subjects(subj)
eng.init_views(*W.initial_views(B.SUBJECTS))
buf = (C.c_uint64 * 8)()
for t in range(B.SETTLE_ROUNDS):
    eng.round(t, ml[t], acts[t])
torch.cuda.synchronize()
assert L.rsf_gossip_merge_prof(buf) == 0, "library not built with RSF_MERGE_PROF=1"
for t in range(B.SETTLE_ROUNDS, rounds):
    eng.round(t, ml[t], acts[t])
torch.cuda.synchronize()
L.rsf_gossip_merge_prof(buf)
v = list(buf)
names = ["setup", "chunk_loads", "chain_walk", "serial", "stores", "total", "waves"]
if len(sys.argv) > 2 and sys.argv[2] == "emit":  # a library built with -DRSF_EMIT_PROF=1
    names = ["rt1_wait", "rt2_wait", "pending_apply", "pick_loop", "materialize", "total", "waves", "stores"]
out = {k: v[i] for i, k in enumerate(names)}
out["share"] = {k: round(v[i] / max(1, v[5]), 3) for i, k in enumerate(names) if k not in ("total", "waves")}
out["cycles_per_wave"] = v[5] / max(1, v[6])
print(json.dumps(out))
