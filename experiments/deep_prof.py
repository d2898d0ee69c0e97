"""Diagnostic only: why emit_run defers members to the deep path and where the deep wave
kernel spends its time, at the bench's configs[1] shape (needs a library built with
-DRSF_DEEP_PROF=1, loaded via RSF_LIB_PATH).  depth: the intent queue's depth; period > 0:
the reference's regime (in-round staggered checker ticks to 4096 every `period` rounds, the
ring sized so nothing expires).
Usage: deep_prof.py [members] [settle] [depth] [period]"""
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
settle = int(sys.argv[2]) if len(sys.argv) > 2 else B.SETTLE_ROUNDS
depth = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
period = int(sys.argv[4]) if len(sys.argv) > 4 else 0
L = lib()
L.rsf_gossip_deep_prof.restype = C.c_int
L.rsf_gossip_deep_prof.argtypes = [C.POINTER(C.c_uint64)]
rounds = settle + 5
cfg = B.gossip_cfg(n, rounds, 1, queue_depth=depth, ring_rounds=rounds)
subj, acts, ml = W.intents_workload(n, B.SUBJECTS, rounds, rate=0.01, seed=B.SEED, prune_frac=B.PRUNE_FRAC)
eng = GossipEngine(cfg)
eng.set_subjects(subj)
eng.init_views(*W.initial_views(B.SUBJECTS))
if period:
    eng.set_checker(period, 4096, 0, 128)
buf = (C.c_uint64 * 80)()
for t in range(settle):
    eng.round(t, ml[t], acts[t])
torch.cuda.synchronize()
assert L.rsf_gossip_deep_prof(buf) == 0, "library not built with RSF_DEEP_PROF=1"
for t in range(settle, rounds):
    eng.round(t, ml[t], acts[t])
torch.cuda.synchronize()
L.rsf_gossip_deep_prof(buf)
v = [int(x) for x in buf]
why = ["empty_head", "pick_len", "pick_key", "exact_empty", "exact_len", "exact_key", "capacity", "tail_bound_tx0"]
ph = ["load", "prune", "take_head", "picks", "store", "fallback_picks", "fallback_store", "fallbacks"]
members = max(1, v[16])
out = {"rounds": rounds - settle, "deferred_per_round": v[16] / (rounds - settle),
       "why_per_round": {k: v[i] / (rounds - settle) for i, k in enumerate(why)},
       "cycles_per_member": v[17] / members,
       "phase_cycles_per_member": {k: v[8 + i] / members for i, k in enumerate(ph)},
       "exact_key_split_per_round": {"crossing_pick_in_leading_run": v[24] / (rounds - settle),
                                     "crossing_pick_is_later_fit": v[25] / (rounds - settle),
                                     "no_tail_item_fits_before_it": v[26] / (rounds - settle)},
       "select_passes_per_select": v[18] / max(1, v[19]), "selects_per_member": v[19] / members,
       "take_head_cycles_per_member": {k: v[20 + i] / members for i, k in enumerate(["count", "select", "gather", "rank_permute"])},
       "crossing_pick_tx0_per_round": v[27] / (rounds - settle), "crossing_pick_tx_ge1_per_round": v[28] / (rounds - settle),
       "recent_mode_per_round": v[29] / (rounds - settle), "recent_relisted_per_round": v[30] / (rounds - settle),
       "queue_items_hist_by_128": {i * 128: v[32 + i] for i in range(32) if v[32 + i]},
       "per_class": {k: {"members_per_round": v[74 + i] / (rounds - settle),
                         "cycles_per_member": v[70 + i] / max(1, v[74 + i])}
                     for i, k in enumerate(["tiny", "small", "middle", "full"])}}
print(json.dumps(out))
