"""configs[3] leg of bench.py (`--workload churn`): a 100k-member cluster with 1%
churn (members fail or leave; a quarter of the failures are force-left with prune)
and a flood of 100 user events (cc 50%) + 10 queries per round, event/query buffers
512, retransmit mult 4.

Two passes over the same seeded workload (the engine is deterministic, so both
passes compute identical rounds):
  timed    : --warmup + --steps rounds, the round only -> node-rounds/s (by default in the
             reference's queue regime: --queue-depth for all three queues, the in-round
             staggered QueueChecker every --check-every rounds, no ring expiry; with
             --queue-depth 0 the bounded 64-slot model)
  delivery : the same rounds plus a dissemination tail with the delivery log on
             (UserEvents handed to the application, base.rs:831-835): for every
             user event originated in the timed window, how many live members
             delivered it, and after how many rounds all of them had (rounds to
             full delivery); plus the coalesced delivery volume of one
             UserEventCoalescer per member (coalesce/user.rs:52-97).
"""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
SEED = 0x5EED5EED
N_DEFAULT = 100_000
EVENTS, QUERIES = int(os.environ.get("RSF_CHURN_EVENTS", 100)), int(os.environ.get("RSF_CHURN_QUERIES", 10))
TAIL = 24  # dissemination rounds after the timed window (delivery pass)


MAX_QUEUE_DEPTH, QUEUE_DEPTH_WARNING = 4096, 128  # options.rs:512 (max_queue_depth), the checker's warning


def churn_cfg(n, s, depth=0, rounds_total=64):
    """depth > 64: the reference's queue regime -- all three queues that deep (register head +
    HBM tail), pruned only by the staggered QueueChecker, and the rumor ring sized so nothing
    expires in `rounds_total` rounds; 0: the bounded 64-slot model with a 2^16-slot ring."""
    from ruserf_amd.gossip import GossipConfig
    ring = 1 << 16
    if depth:
        per_round = s * 4 + EVENTS + QUERIES
        ring = 1 << max(16, (per_round * rounds_total - 1).bit_length())
    return GossipConfig(n_members=n, n_subjects=s, queue_cap=64, event_buffer_size=512, query_buffer_size=512,
                        slot_k=16, fanout=3, gossip_limit=1400, gossip_overhead=2, retransmit_mult=4, max_refute=4,
                        max_rumors=ring, seed=SEED, queue_depth=(depth, depth, depth) if depth else None)


def _engine(n, rounds_total, depth=0, check_every=0):
    from ruserf_amd import workload as W
    from ruserf_amd.gossip import GossipEngine
    subj, acts, ml = W.churn_workload(n, rounds_total, events_per_round=EVENTS, queries_per_round=QUERIES,
                                      seed=SEED)
    eng = GossipEngine(churn_cfg(n, len(subj), depth, rounds_total), device=torch.cuda.current_device())
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.set_subjects(subj)
    eng.init_views(*W.initial_views(len(subj)))
    if depth and check_every:
        # each member's QueueChecker on its own phase (member id mod check_every), in the rounds
        eng.set_checker(check_every, MAX_QUEUE_DEPTH, 0, QUEUE_DEPTH_WARNING)
    return eng, subj, acts, ml


def run_churn(args, rank, world):
    from ruserf_amd.coalesce import MEMBER_EVENT_DTYPE, USER_EVENT_DTYPE, MemberEventCoalescer, coalesce_user_events
    from ruserf_amd.gossip import ACT_USER_EVENT, DELIVERY_MEMBER_EVENT, DELIVERY_USER_EVENT, E_QUEUE_PRUNE
    n = args.members or N_DEFAULT
    timed_rounds = args.warmup + args.steps
    rounds_total = timed_rounds + TAIL
    depth = getattr(args, "queue_depth", 0) or 0
    check_every = (getattr(args, "check_every", 0) or 0) if depth else 0
    # ---- timed pass
    eng, subj, acts, ml = _engine(n, rounds_total, depth, check_every)
    for t in range(args.warmup):
        eng.round(t, ml[t], acts[t])
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    merged0 = eng.merged_total()
    eng.set_profiling(True)
    t0 = time.perf_counter()
    for t in range(args.warmup, timed_rounds):
        eng.round(t, ml[t], acts[t])
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    wall = time.perf_counter() - t0
    phase_ms, nr = eng.phase_times()
    merged = eng.merged_total() - merged0
    eng.set_profiling(False)
    regime = None
    if depth:
        ql = eng.queue_lengths().astype(np.int64)
        regime = {"what": "the reference's queue regime: all three queues " + str(depth) + " deep, pruned only by "
                          "each member's QueueChecker (every " + str(check_every) + " rounds on its own phase, to "
                          + str(MAX_QUEUE_DEPTH) + "), no rumor-ring expiry",
                  "queue_items_after_window": {q: {"mean": float(ql[:, i].mean()), "max": int(ql[:, i].max())}
                                               for i, q in enumerate(["intent", "query", "event"])},
                  "bounded_pruned_total": int(eng.pruned().astype(np.uint64).sum()),
                  "expired_total": int(eng.expired().astype(np.uint64).sum()),
                  "deferred_per_round_by_class": dict(zip(["tiny", "small", "middle", "full"],
                                                          (eng.deep_class_stats() / max(1, timed_rounds)).tolist()))}
    eng.close()
    if world > 1:  # independent replicas (configs[3] is a one-GPU cluster)
        t_ = torch.tensor([wall], dtype=torch.float64, device="cuda")
        torch.distributed.all_reduce(t_, op=torch.distributed.ReduceOp.MAX)
        wall = float(t_[0])
    # ---- delivery pass (untimed), the same rounds with the delivery log
    eng, subj, acts, ml = _engine(n, rounds_total, depth, check_every)
    eng.set_delivery_log(768)
    # member events: one MemberEventCoalescer per member over its stream, a quantum per round
    mcoal = MemberEventCoalescer(n, len(subj))
    mev_in = mev_out = 0
    dead = np.zeros(n, dtype=bool)
    per_round = []
    for t in range(rounds_total):
        eng.round(t, ml[t], acts[t])
        for e in ml[t]:
            if e["set_alive"] == 0:
                dead[subj[e["subject"]]] = True
            elif e["set_alive"] == 1:
                dead[subj[e["subject"]]] = False
        d = eng.deliveries()
        me = d[d["kind"] == DELIVERY_MEMBER_EVENT]
        if len(me):
            mev = np.zeros(len(me), MEMBER_EVENT_DTYPE)
            mev["group"], mev["node"], mev["type"] = me["member"], me["key"], me["ltime"]
            mev_in += len(me)
            mev_out += len(mcoal.flush(mev))
        per_round.append(d[d["kind"] == DELIVERY_USER_EVENT])
    mcoal.close()
    st = eng.members()
    pruned = int(eng.pruned().astype(np.uint64).sum())
    err_other = int(np.count_nonzero(st["err"] & ~np.uint32(E_QUEUE_PRUNE)))
    err_bits = {name: int(np.count_nonzero(st["err"] & np.uint32(bit))) for name, bit in
                [("event_slot_full", 1), ("query_slot_full", 2), ("refute_full", 4), ("stage_full", 8),
                 ("queue_prune", 16), ("delivery_log_full", 32)]}
    eng.close()
    live = int(np.count_nonzero(~dead))
    # events originated in the timed window, by key; deliveries per round
    keys, born = [], []
    for t in range(args.warmup, timed_rounds):
        a = acts[t]
        ue = a[a["act"] == ACT_USER_EVENT]
        keys.append(ue["key"])
        born.append(np.full(len(ue), t))
    keys = np.concatenate(keys)
    born = np.concatenate(born)
    order = np.argsort(keys)
    keys, born = keys[order], born[order]
    cum = np.zeros(len(keys), dtype=np.int64)
    full_at = np.full(len(keys), -1, dtype=np.int64)
    for t, d in enumerate(per_round):
        if len(d) == 0:
            continue
        idx = np.searchsorted(keys, d["key"])
        ok = (idx < len(keys)) & (keys[np.minimum(idx, len(keys) - 1)] == d["key"])
        cum += np.bincount(idx[ok], minlength=len(keys))
        newly = (full_at < 0) & (cum >= live)
        full_at[newly] = t
    reached = full_at >= 0
    lat = (full_at - born)[reached] + 1  # rounds from origination to the last delivery, inclusive
    # the coalescer over each member's cc deliveries of the whole run (one coalescer per member)
    d = np.concatenate(per_round)
    d = d[d["cc"] == 1]
    d = d[np.argsort(d["member"], kind="stable")]
    ev = np.zeros(len(d), USER_EVENT_DTYPE)
    ev["group"] = d["member"]
    ev["name"] = (d["key"] >> np.uint64(32)).astype(np.uint32)
    ev["ltime"] = d["ltime"]
    ev["payload"] = d["key"] & np.uint64(0xFFFFFFFF)
    coalesced = len(coalesce_user_events(ev)) if len(ev) else 0
    avg = [x / max(1, nr) for x in phase_ms]
    from bench_gossip import B_MERGE, HBM_PEAK_GBS
    records = merged / max(1, args.steps)
    achieved = records * B_MERGE / (avg[3] / 1e3) / 1e9 if avg[3] else 0.0
    names = ["begin (memberlist+refute+originate)", "peers+group sort", "emit_kernel", "merge_kernel"]
    return {
        "metric": "gossip node-rounds/s", "value": n * args.steps * max(1, world) / wall, "unit": "node-rounds/s",
        "ms_per_step": wall / args.steps * 1e3, "dtype": "u64",
        "scaling": "weak",
        "config": {"workload": f"BASELINE configs[3]: {n} members, 1% churn ({len(subj)} subjects fail or leave, "
                               f"25% of failures force-left with prune), {EVENTS} user events (cc 50%) + {QUERIES} "
                               f"queries per round, event/query buffers 512, retransmit mult 4, fanout 3, "
                               + (f"the reference's queue regime (queues {depth} deep, staggered checker every "
                                  f"{check_every} rounds to {MAX_QUEUE_DEPTH})" if depth else
                                  "bounded 64-slot queues (model point)"),
                   "members": n, "members_per_gpu": n, "queue_depth": depth or 64,
                   "parallelism": "one cluster per GPU" + (f" ({world} independent replicas)" if world > 1 else "")},
        "queue_regime": regime,
        "phases_ms_per_round": dict(zip(names, avg)),
        "merges_per_s": merged / wall, "records_per_round_per_gpu": records,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": "merge_kernel",
                     "bytes_model": "SURVEY 8(d): B_merge = 64 B per merged record", "bytes_per_unit": B_MERGE,
                     "units_per_launch": records, "bytes_per_launch": records * B_MERGE,
                     "avg_launch_ms": avg[3]},
        "delivery": {
            "events_tracked": int(len(keys)), "rounds_observed_after_window": TAIL,
            "live_members_at_end": live,
            "fully_delivered_frac": float(reached.mean()) if len(keys) else None,
            "mean_delivered_frac": float(np.mean(np.minimum(cum, live) / live)) if len(keys) else None,
            "rounds_to_full_delivery": {"median": float(np.median(lat)) if len(lat) else None,
                                        "p90": float(np.percentile(lat, 90)) if len(lat) else None,
                                        "max": int(lat.max()) if len(lat) else None},
            "cc_deliveries": int(len(ev)), "after_coalescing": int(coalesced),
            "member_events": int(mev_in), "member_events_after_coalescing": int(mev_out),
            "queue_pruned_total": pruned, "error_members_other": err_other, "members_by_error_bit": err_bits,
        },
    }


def cpu_baseline_churn(args, seconds_target=10.0):
    """The oracle's threaded round (orc_world_round_mt) on the same configs[3] workload:
    it fits the CPU at full size, so the sample is the first rounds of the same run."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import gossip_harness as H  # test infrastructure: checker / CPU baseline only
    from bench import cpu_info, cpu_threads
    from ruserf_amd import workload as W
    n = args.members or N_DEFAULT
    th = cpu_threads()
    rounds_total = args.warmup + args.steps + TAIL
    subj, acts, ml = W.churn_workload(n, rounds_total, events_per_round=EVENTS, queries_per_round=QUERIES,
                                      seed=SEED)
    depth = getattr(args, "queue_depth", 0) or 0
    check_every = (getattr(args, "check_every", 0) or 0) if depth else 0
    w = H.oracle_world(churn_cfg(n, len(subj), depth, rounds_total), subj, W.initial_views(len(subj)))
    if depth and check_every:
        H.L.orc_world_set_checker(C.byref(w), MAX_QUEUE_DEPTH, 0, QUEUE_DEPTH_WARNING, check_every)
    t = 0
    for _ in range(args.warmup):
        H.oracle_round(w, t, ml[t], acts[t], threads=th)
        t += 1
    done, spent = 0, 0.0
    while spent < seconds_target and t < args.warmup + args.steps:
        t0 = time.perf_counter()
        H.oracle_round(w, t, ml[t], acts[t], threads=th)
        spent += time.perf_counter() - t0
        done += 1
        t += 1
    H.L.orc_world_free(C.byref(w))
    return {"value": n * done / spent, "unit": "node-rounds/s", "cores": th, "kind": "port",
            "sample": f"oracle configs[3] rounds {args.warmup}..{t - 1} ({done} rounds, {spent:.1f}s) of the same "
                      f"workload and queue configuration (depth {depth or 64}) on {th} threads; {cpu_info()}"}
