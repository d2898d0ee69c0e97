"""Gossip-round leg of bench.py (metric: node-rounds/s, BASELINE configs[1]/[2]).

A node-round = one member processing one gossip round: select
k=3 live peers, drain its intent/query/event queues under the byte budget
(b = 8 intents per target), emit, receive and merge its inbound records in
canonical order, update its Lamport clocks.
"""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))

SEED = 0x5EED5EED
SUBJECTS = 4096
SETTLE_ROUNDS = 12   # setup: bring the cluster to gossip steady state (queues saturated) before timing
# the reference's queue regime (deep queues): QueueChecker ticks every queue_check_interval
# = 30 s (options.rs:512) at memberlist's LAN gossip interval of 200 ms = 150 rounds, each
# pruning every queue to max_queue_depth 4096 (base.rs:720-760); settled past two ticks
CHECK_EVERY = 150
SETTLE_STEADY = 330
MAX_QUEUE_DEPTH = 4096
QUEUE_DEPTH_WARNING = 128
# fraction of force_leaves issued with prune (remove_failed_node_prune); RSF_PRUNE_FRAC overrides
PRUNE_FRAC = float(os.environ.get("RSF_PRUNE_FRAC", 0.1))
HBM_PEAK_GBS = 8000.0


def gossip_cfg(n_total, rounds_total, world, shard=None, queue_cap=64, queue_depth=0, ring_rounds=64,
               retransmit_mult=4):
    """queue_depth > queue_cap: the intent queue (the only one this workload fills) is that
    deep -- register head + HBM tail, pruned only by the QueueChecker as the reference's
    (max_queue_depth 4096); the query / event queues stay at queue_cap (always empty here).
    ring_rounds: the rumor ring holds at least that many rounds of rumor blocks in one
    generation, so no queued item expires within that many rounds (the reference never
    expires one: ring_rounds >= the run's rounds makes the model's ring invisible)."""
    from ruserf_amd.gossip import GossipConfig
    # rumor ring: a power of two holding >= ring_rounds rounds of rumor blocks (ids recycle after that)
    per_round = SUBJECTS * 4 + int(round(n_total * 0.01))
    ring = 1 << max(10, (per_round * max(64, ring_rounds) - 1).bit_length())
    return GossipConfig(n_members=n_total, n_subjects=SUBJECTS, shard=shard, queue_cap=queue_cap, event_buffer_size=512,
                        query_buffer_size=512, slot_k=1, fanout=3, gossip_limit=8 * 24, gossip_overhead=2,
                        retransmit_mult=retransmit_mult, max_refute=4, max_rumors=ring, seed=SEED,
                        queue_depth=(queue_depth, 0, 0) if queue_depth > queue_cap else None)


# B_merge = 16 (record read) + 16 (view entry read) + 16 (view entry write)
# + 16 (clock r/w, counted once per record as an upper bound) = 64 B per merged record
B_MERGE = 64


def kernel_bytes(qcap, senders, records, fanout=3):
    """Algorithmic HBM bytes per launch.

    `roofline` (the driver line) prices the merge kernel with SURVEY §8(d)'s model
    only: B_MERGE = 64 B per merged record.  The extended model (reported beside it)
    adds what this engine's queue model must also move (intents only:
    the query/event queues stay empty):
    emit  : per live sender its peers + group slots (8 B per peer), the intent queue read
            and written back (16 B per slot: rumor id, seq, transmits|len, decoration; it
            is re-ranked after every pick), its pending re-queues read (12 B each, about
            one per record merged), and per record the rumor id + decoration written
            (8 B), per group its count (4 B)
    merge : B_MERGE per record plus the re-queue appended to the receiver's pending list
            (12 B; the merge no longer reads or writes the queues)."""
    queue_rw = 2 * qcap * 16
    emit = senders * (fanout * 8 + queue_rw + fanout * 4) + records * (8 + 12)
    merge_s8d = records * B_MERGE
    merge_ext = merge_s8d + records * 12
    return emit, merge_s8d, merge_ext


def run_gossip(args, rank, world):
    from ruserf_amd import workload as W
    from ruserf_amd.dist import ShardedGossip
    from ruserf_amd.gossip import GossipEngine
    per = args.members
    n = per * world
    depth = getattr(args, "queue_depth", 0) or 0
    # QueueChecker ticks in the round loop (0: none), staggered: each member's checker runs on
    # its own timer (base.rs:703-735), member m ticking in the rounds r with r % K == m % K,
    # so every round carries 1/K of the ticks (the prune included in the timed steps at its
    # true rate) and the queues cycle between max_queue_depth and what K rounds add; the ring
    # sized so no queued item expires during the run
    check_every = getattr(args, "check_every", 0) or 0
    settle = (SETTLE_STEADY if check_every else SETTLE_ROUNDS) if args.settle is None else args.settle
    rounds_total = settle + args.warmup + args.steps
    # the rumor ring: sized for the whole run in the queue regime (no queued item expires, as in
    # the reference); --ring-rounds overrides it (an A/B of the merge's rumor-body gather against
    # a ring small enough for the MALL -- items then expire, counted in expired_whole_run)
    ring_rounds = getattr(args, "ring_rounds", None) or (rounds_total if check_every else 64)
    cfg = gossip_cfg(n, rounds_total, world, queue_cap=args.queue_cap, queue_depth=depth, ring_rounds=ring_rounds)
    subj, acts, ml = W.intents_workload(n, SUBJECTS, rounds_total, rate=0.01, seed=SEED, prune_frac=PRUNE_FRAC)
    views = W.initial_views(SUBJECTS)
    stream = torch.cuda.current_stream()
    sharded = not (world == 1 and os.environ.get("RSF_FORCE_SHARDED") != "1")
    if not sharded:
        eng = GossipEngine(cfg, device=torch.cuda.current_device())
        eng.set_stream(stream.cuda_stream)
        step_fn = lambda t: eng.round(t, ml[t], acts[t])  # noqa: E731
    else:
        sg = ShardedGossip(cfg, rank, world, device=torch.cuda.current_device())
        eng = sg.eng
        step_fn = lambda t: sg.round(t, ml[t], acts[t])  # noqa: E731
    eng.set_subjects(subj)
    eng.init_views(*views)
    if check_every:
        # the staggered ticks inside the rounds: round r ticks the members with id = r mod K,
        # between its emission and its merge
        eng.set_checker(check_every, MAX_QUEUE_DEPTH, 0, QUEUE_DEPTH_WARNING)

    def step_settle(t_):
        step_fn(t_)

    t = 0
    for _ in range(settle + args.warmup):
        step_settle(t)
        t += 1
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    merged0 = eng.merged_total()
    # as of each member's last emission (no flush): the timed rounds' emissions apply
    # exactly the timed rounds' worth of pending re-queues
    pruned0 = eng.pruned_total(flush=False)
    deep0 = eng.deep_stats()[0] if depth else 0
    cls0 = eng.deep_class_stats() if depth else None
    if check_every:
        eng.checker_stats(reset=True)
    eng.set_profiling(True)
    if sharded:
        sg.set_timing(True)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step_fn(t)
        t += 1
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    wall = time.perf_counter() - t0
    # multi-GPU path: no bucket overflowed and every record reached its shard (read after timing)
    exchange_ok = sg.check() if sharded else None
    exchange_ms = sg.exchange_times() if sharded else None
    phase_ms, nr = eng.phase_times()
    merged = eng.merged_total() - merged0
    pruned = eng.pruned_total(flush=False) - pruned0
    deep_members = (eng.deep_stats()[0] - deep0) if depth else None
    regime = None
    if check_every:
        occ = eng.checker_occupancy()
        cst = eng.checker_stats()
        h, b = occ["hist"][0].astype(np.int64), occ["bin"]
        cum = np.cumsum(h)
        q = lambda f: int((np.searchsorted(cum, f * cum[-1]) + 1) * b)  # noqa: E731  (upper edge of the bin)
        ticked = int(cum[-1])
        ql = eng.queue_lengths()[:, 0].astype(np.int64)
        regime = {"what": "the reference's queue regime: each member's QueueChecker ticks every check_every rounds "
                          "(queue_check_interval 30 s / gossip interval 200 ms) on its own phase (member id mod "
                          "check_every), pruning its queues to max_queue_depth; nothing dropped in between "
                          "(bounded_pruned = 0), no rumor-ring expiry",
                  "check_every_rounds": check_every, "max_queue_depth": MAX_QUEUE_DEPTH,
                  "intent_queue_capacity": cfg.depths()[0], "settle_rounds": settle,
                  "ticks_in_timed_window": ticked,
                  "intent_queue_items_after_window": {"mean": float(ql.mean()), "p50": int(np.percentile(ql, 50)),
                                                      "p99": int(np.percentile(ql, 99)), "max": int(ql.max()),
                                                      "min": int(ql.min())},
                  "occupancy_at_ticks_in_window": {"members_ticked": ticked,
                                                   "mean": float(cst["queued"][0]) / max(1, ticked),
                                                   "p50_upper": q(0.5), "p99_upper": q(0.99),
                                                   "max": int(occ["max"][0]), "bin": b},
                  "pruned_per_tick": float(cst["pruned"][0]) / max(1, ticked),
                  "pruned_per_round": float(cst["pruned"][0]) / args.steps,
                  "members_over_warning_in_window": int(cst["warn"][0]),
                  "expired_whole_run": int(eng.expired().sum()),
                  "rumor_ring_slots": int(cfg.max_rumors), "ring_rounds": int(ring_rounds),
                  "deferred_per_round_by_class": dict(zip(["tiny", "small", "middle", "full"],
                                                          ((eng.deep_class_stats() - cls0) / args.steps).tolist()))
                  if depth else None}
    st = eng.members()
    from ruserf_amd.gossip import E_QUEUE_PRUNE
    # capacity errors other than the bounded queue's counted prunes (reported separately)
    err_members = int(np.count_nonzero(st["err"] & ~np.uint32(E_QUEUE_PRUNE)))
    qprune_members = int(np.count_nonzero(st["err"] & np.uint32(E_QUEUE_PRUNE)))
    eng.set_profiling(False)
    canaries_ok = all(eng.cub_canaries())  # no hipCUB call wrote past its temporary storage
    if world > 1:
        dev = "cpu" if torch.distributed.get_backend() == "gloo" else "cuda"
        t_ = torch.tensor([wall, float(merged), float(err_members), float(pruned), float(qprune_members),
                           float(bool(exchange_ok))], dtype=torch.float64, device=dev)
        mx = t_.clone()
        torch.distributed.all_reduce(mx, op=torch.distributed.ReduceOp.MAX)
        torch.distributed.all_reduce(t_)
        wall, merged_all, err_all, pruned_all, qpm_all = float(mx[0]), float(t_[1]), float(t_[2]), float(t_[3]), \
            float(t_[4])
        exchange_ok = int(t_[5]) == world  # every rank's buckets held
    else:
        merged_all, err_all, pruned_all, qpm_all = float(merged), float(err_members), float(pruned), \
            float(qprune_members)
    eng.close()  # free the shard's HBM before bench.py's next leg
    node_rounds = n * args.steps
    avg = [x / max(1, nr) for x in phase_ms]  # ms per round per phase
    names = ["begin (memberlist+refute+originate)", "peers+group sort", "emit_kernel" + ("+exchange" if world > 1 else ""),
             "merge_kernel"]
    senders = per
    records = merged / max(1, args.steps)  # records per round on this shard
    emit_b, merge_b, merge_ext = kernel_bytes(cfg.queue_cap, senders, records)
    # the dominant kernel is the merge (phase 3); the roofline prices it with §8(d)'s bytes
    dom = 3
    achieved = merge_b / (avg[dom] / 1e3) / 1e9
    achieved_ext = merge_ext / (avg[dom] / 1e3) / 1e9
    return {
        "metric": "gossip node-rounds/s", "value": node_rounds / wall, "unit": "node-rounds/s",
        "ms_per_step": wall / args.steps * 1e3, "dtype": "u64",
        "config": {"workload": f"gossip rounds, {n} members ({per}/GPU), fanout k=3, {SUBJECTS} tracked subjects, "
                               f"1% of members originate a join/leave intent per round, member-state merge + "
                               f"Lamport clocks, "
                               + (f"the reference's queue regime (intent queue {cfg.depths()[0]} deep, each member's "
                                  f"QueueChecker pruning to {MAX_QUEUE_DEPTH} every {check_every} rounds on its own "
                                  f"phase, inside the timed rounds; settled {settle} rounds) "
                                  if check_every else f"bounded {cfg.queue_cap}-slot queues (model point) ")
                               + ("(BASELINE configs[2] shard: 2M members/GPU, 16M at 8 GPUs)" if per == 2_000_000
                                  else "(BASELINE configs[1]: 1M members on one MI355X)" if per == 1_000_000 and world == 1
                                  else "(1M members per GPU, weak scaling)" if per == 1_000_000 else "(custom size)"),
                   "members": n, "members_per_gpu": per, "fanout": 3, "items_per_target": 8,
                   "queue_cap_per_queue": cfg.queue_cap, "subjects": SUBJECTS,
                   "intent_queue_depth": cfg.depths()[0],
                   "record_slots_per_group": min(3 * cfg.queue_cap, cfg.gossip_limit // (cfg.gossip_overhead + 18)),
                   "settle_rounds": settle, "parallelism": f"members sharded x{world}"
                   + (" (multi-GPU code path forced)" if world == 1 and os.environ.get("RSF_FORCE_SHARDED") == "1"
                      else "")},
        "merges_per_s": merged_all / wall,
        "records_per_round_per_gpu": records,
        "error_members": err_all,
        "exchange_ok": exchange_ok,
        "cub_canaries_intact": canaries_ok,
        # the bounded queue model (queue_cap slots) drops live items when full; counted, not silent
        "queue_pruned_per_round": pruned_all / args.steps,
        "queue_regime": regime,
        "queue_pruned_per_merged_record": pruned_all / max(1.0, merged_all),
        "queue_prune_members": qpm_all,
        # deep queues: members per round whose emission needed the tail (emit_deep_wave_kernel)
        "deep_path_members_per_round": (deep_members / args.steps) if deep_members is not None else None,
        "phases_ms_per_round": dict(zip(names, avg)),
        # multi-GPU path: device time of the round's collectives (inside the phases above)
        "collectives_ms_per_round": exchange_ms,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": names[dom],
                     "bytes_model": "SURVEY 8(d): B_merge = 64 B per merged record",
                     "bytes_per_unit": B_MERGE, "units_per_launch": records,
                     "bytes_per_launch": merge_b, "avg_launch_ms": avg[dom],
                     "extended": {"bytes_per_launch": merge_ext, "achieved": achieved_ext,
                                  "frac": achieved_ext / HBM_PEAK_GBS,
                                  "model": "B_merge per record + its re-queue appended to the "
                                           "receiver's pending list (12 B)"},
                     "emit_kernel": {"avg_launch_ms": avg[2], "bytes_per_launch": emit_b,
                                     "achieved": emit_b / (avg[2] / 1e3) / 1e9 if avg[2] else None}},
    }


def cpu_baseline_gossip_deep(args, seconds_target=12.0, n=5_000):
    """The oracle's round in the line's queue regime and at its occupancy, on a bounded sample:
    n members, the intent queue as deep as the engine's, the staggered QueueChecker (every
    CHECK_EVERY rounds to MAX_QUEUE_DEPTH) and the ring sized so nothing expires, settled
    SETTLE_STEADY rounds -- as the GPU line -- so the queues hold 4-6k items; then timed on all
    the box's threads and on one.  The retransmit limit is the line's (28 = 4 x 7 digits at
    1M members): at n members the multiplier is scaled to give the same limit.  The oracle's
    queue is an array scanned per pick (memberlist's TransmitLimitedQueue is a btree); the CPU
    figure is the restatement's."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import gossip_harness as H  # test infrastructure: checker / CPU baseline only
    from bench import cpu_info, cpu_threads
    from ruserf_amd import workload as W
    th = cpu_threads()
    settle = SETTLE_STEADY
    rounds_total = settle + 72
    L = H.L
    digits = lambda x: len(str(int(x)))  # noqa: E731  (ceil(log10(x + 1)) for x >= 1)
    limit = 4 * digits(max(1, args.members))
    mult = max(1, round(limit / digits(n)))
    cfg = gossip_cfg(n, rounds_total, 1, queue_cap=64, queue_depth=args.queue_depth, ring_rounds=rounds_total,
                     retransmit_mult=mult)
    subj, acts, ml = W.intents_workload(n, SUBJECTS, rounds_total, rate=0.01, seed=SEED, prune_frac=PRUNE_FRAC)
    w = H.oracle_world(cfg, subj, W.initial_views(SUBJECTS))
    t = 0
    L.orc_world_set_checker(C.byref(w), MAX_QUEUE_DEPTH, 0, QUEUE_DEPTH_WARNING, CHECK_EVERY)

    def rnd(threads):
        H.oracle_round(w, t, ml[t], acts[t], threads=threads)
    t_settle = time.perf_counter()
    for _ in range(settle):
        rnd(th)
        t += 1
    t_settle = time.perf_counter() - t_settle

    def timed(threads, budget, max_rounds):
        nonlocal t
        done, spent = 0, 0.0
        while spent < budget and done < max_rounds and t < rounds_total:
            t0 = time.perf_counter()
            rnd(threads)
            spent += time.perf_counter() - t0
            done += 1
            t += 1
        return done, spent
    done_mt, spent_mt = timed(th, seconds_target, 60)
    done_1, spent_1 = timed(1, seconds_target / 2, 10)
    hw = H.world_width(w)
    ql = (H.O.arr(w.q_rumor, n * 3 * w.qcap, np.uint32).reshape(n, 3, w.qcap)[:, 0, :hw] != 0xFFFFFFFF).sum(axis=1)
    L.orc_world_free(C.byref(w))
    return {"value": n * done_mt / spent_mt, "unit": "node-rounds/s", "cores": th, "kind": "port",
            "value_1thread": n * done_1 / spent_1,
            "cpu_model": cpu_info(),
            "queue_items": {"mean": float(ql.mean()), "p99": int(np.percentile(ql, 99)), "max": int(ql.max())},
            "sample": f"oracle gossip rounds (orc_world_round_mt), {n} members, {SUBJECTS} subjects, the line's workload, "
                      f"queue regime and depth ({cfg.depths()[0]}; staggered checker every {CHECK_EVERY} rounds to "
                      f"{MAX_QUEUE_DEPTH}; retransmit limit {limit}), settled {settle} rounds ({t_settle:.0f}s, not "
                      f"timed) to intent queues of mean {ql.mean():.0f} / p99 {np.percentile(ql, 99):.0f} items; "
                      f"{done_mt} rounds on {th} threads ({spent_mt:.1f}s), {done_1} rounds on 1 thread "
                      f"({spent_1:.1f}s); {cpu_info()}"}


def cpu_baseline_gossip(args, seconds_target=10.0, n=200_000):
    """The oracle's round (the C restatement of the same path) on a bounded sample:
    n members, the same subject count and workload, settled, then timed with all the
    box's threads (orc_world_round_mt: member loops partitioned over pthreads, results
    identical to one thread) and with one thread (both rates + the CPU)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import gossip_harness as H  # test infrastructure: checker / CPU baseline only
    from bench import cpu_info, cpu_threads
    from ruserf_amd import workload as W
    th = cpu_threads()
    rounds_total = SETTLE_ROUNDS + 40
    cfg = gossip_cfg(n, rounds_total, 1, queue_cap=getattr(args, "queue_cap", 64))
    subj, acts, ml = W.intents_workload(n, SUBJECTS, rounds_total, rate=0.01, seed=SEED, prune_frac=PRUNE_FRAC)
    w = H.oracle_world(cfg, subj, W.initial_views(SUBJECTS))
    t = 0
    for _ in range(SETTLE_ROUNDS):
        H.oracle_round(w, t, ml[t], acts[t], threads=th)
        t += 1

    def timed(threads, budget, max_rounds):
        nonlocal t
        done, spent = 0, 0.0
        while spent < budget and done < max_rounds and t < rounds_total:
            t0 = time.perf_counter()
            rnd(threads)
            spent += time.perf_counter() - t0
            done += 1
            t += 1
        return done, spent
    done_mt, spent_mt = timed(th, seconds_target, 30)
    done_1, spent_1 = timed(1, seconds_target / 2, 4)
    H.L.orc_world_free(C.byref(w))
    return {"value": n * done_mt / spent_mt, "unit": "node-rounds/s", "cores": th, "kind": "port",
            "value_1thread": n * done_1 / spent_1,
            "cpu_model": cpu_info(),
            "sample": f"oracle gossip rounds (orc_world_round_mt), {n} members, {SUBJECTS} subjects, same workload "
                      f"settled {SETTLE_ROUNDS} rounds; {done_mt} rounds on {th} threads ({spent_mt:.1f}s), "
                      f"{done_1} rounds on 1 thread ({spent_1:.1f}s); {cpu_info()}"}
