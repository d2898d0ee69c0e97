"""Diagnostic: per-round cost of the multi-GPU split without the interconnect.
Two 1M-member shard contexts in ONE process on one GPU (views 2 x 64 GB), the
all-reduce / all-to-all replaced by device copies; each shard's work is timed
separately and compared with a single 1M-member context running the same
per-GPU workload (the N=1 bench)."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench_gossip as B  # noqa: E402
from ruserf_amd import gossip as G  # noqa: E402
from ruserf_amd import workload as W  # noqa: E402
from ruserf_amd.dist import hbm_tensor  # noqa: E402

per = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
world = 2
n = per * world
rounds = B.SETTLE_ROUNDS + 6
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
cfg = B.gossip_cfg(n, rounds, world)
subj, acts, ml = W.intents_workload(n, B.SUBJECTS, rounds, rate=0.01, seed=B.SEED)
shards = []
for r in range(world):
    e = G.GossipEngine(G.GossipConfig(**{**cfg.__dict__, "shard": (r * per, (r + 1) * per)}))
    e.set_stream(stream.cuda_stream)
    e.set_subjects(subj)
    e.init_views(*W.initial_views(B.SUBJECTS))
    shards.append(e)
recv = [torch.empty(e.send_buffer()[1], dtype=torch.int64, device="cuda") for e in shards]
times = {"begin": [], "emit": [], "exchange": [], "merge_runs": []}


def ev():
    e = torch.cuda.Event(enable_timing=True)
    e.record(stream)
    return e


for t in range(rounds):
    e0 = ev()
    for e in shards:
        e.round_begin(t, ml[t], acts[t])
    e1 = ev()
    blocks = [hbm_tensor(*e.rumor_block()[:1], e.rumor_block()[1] // 8) for e in shards]
    tot = blocks[0] + blocks[1]
    for b in blocks:
        b.copy_(tot)
    e2 = ev()
    counts = [e.round_emit(world) for e in shards]
    e3 = ev()
    sends = [hbm_tensor(e.send_buffer()[0], int(c.sum())) for e, c in zip(shards, counts)]
    rcs = []
    for dst in range(world):
        parts, rc = [], []
        for src in range(world):
            off = int(counts[src][:dst].sum())
            parts.append(sends[src][off: off + int(counts[src][dst])])
            rc.append(int(counts[src][dst]))
        torch.cat(parts, out=recv[dst][: sum(rc)])
        rcs.append(rc)
    e4 = ev()
    for dst, e in enumerate(shards):
        e.round_merge_runs(recv[dst].data_ptr(), rcs[dst])
    e5 = ev()
    torch.cuda.synchronize()
    if t >= B.SETTLE_ROUNDS:
        times["begin"].append(e0.elapsed_time(e1) / world)
        times["emit"].append(e2.elapsed_time(e3) / world)
        times["exchange"].append((e1.elapsed_time(e2) + e3.elapsed_time(e4)) / world)
        times["merge_runs"].append(e4.elapsed_time(e5) / world)
out = {k: float(np.mean(v)) for k, v in times.items()}
out["per_shard_total_ms"] = sum(out.values())
out["members_per_shard"] = per
print(json.dumps(out))
