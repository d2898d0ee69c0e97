"""Push/pull anti-entropy leg of bench.py: every member runs
one push/pull exchange (memberlist's periodic pushPull) with a random partner —
a perfect matching, both directions — i.e. SerfDelegate::local_state on both
sides then merge_remote_state (core/src/serf/delegate.rs:376-554) on both.
State comes from settled gossip rounds of BASELINE configs[1] (1M members,
4096 tracked subjects, intents) plus a user-event stream so the event buffers
are live.  One step = one push/pull round over all members."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
SEED = 0x5EED5EED
SUBJECTS = 4096
SETTLE_ROUNDS = 10
HBM_PEAK_GBS = 8000.0
BATCH = 1 << 16  # receivers per push_pull call (snapshot slab ~5 GB)


def pp_cfg(n, rounds):
    from ruserf_amd.gossip import GossipConfig
    per_round = SUBJECTS * 4 + int(round(n * 0.01)) + 256
    return GossipConfig(n_members=n, n_subjects=SUBJECTS, queue_cap=64, event_buffer_size=512,
                        query_buffer_size=512, slot_k=1, fanout=3, gossip_limit=8 * 24, gossip_overhead=2,
                        retransmit_mult=4, max_refute=4, max_rumors=1 << max(10, (per_round * rounds - 1).bit_length()), seed=SEED)


def state_bytes(cfg):
    """one member's local_state as the merge reads it: view S x 16 B, event buffer
    (ltime 8 + count 4 + slot_k x 8 per slot), three clocks"""
    return cfg.n_subjects * 16 + cfg.event_buffer_size * (12 + 8 * cfg.slot_k) + 24


def workload(n, rounds):
    from ruserf_amd import workload as W
    from ruserf_amd.gossip import ACT_USER_EVENT, ACTION_DTYPE
    subj, acts, ml = W.intents_workload(n, SUBJECTS, rounds, rate=0.01, seed=SEED)
    rng = np.random.Generator(np.random.Philox(SEED + 1))
    out = []
    for a in acts:  # add 256 user events per round from members not otherwise acting
        free = np.setdiff1d(rng.choice(n, size=1024, replace=False).astype(np.uint32), a["member"])[:256]
        e = np.zeros(len(free), ACTION_DTYPE)
        e["member"], e["act"], e["name_len"], e["payload_len"] = free, ACT_USER_EVENT, 8, 32
        e["key"] = (rng.integers(0, 16, size=len(free)).astype(np.uint64) << np.uint64(32)) | \
            np.arange(len(free), dtype=np.uint64)
        b = np.concatenate([a, e])
        out.append(b[np.argsort(b["member"], kind="stable")])
    return subj, out, ml


def run_pushpull(args, rank, world):
    from ruserf_amd import workload as W
    from ruserf_amd.gossip import PP_PAIR_DTYPE, GossipEngine
    assert world == 1, "push/pull bench is single-GPU (replicas only)"
    n = args.members
    cfg = pp_cfg(n, SETTLE_ROUNDS)
    subj, acts, ml = workload(n, SETTLE_ROUNDS)
    stream = torch.cuda.current_stream()
    eng = GossipEngine(cfg, device=torch.cuda.current_device())
    eng.set_stream(stream.cuda_stream)
    eng.set_subjects(subj)
    eng.init_views(*W.initial_views(SUBJECTS))
    for t in range(SETTLE_ROUNDS):
        eng.round(t, ml[t], acts[t])
    rng = np.random.Generator(np.random.Philox(SEED + 2))
    steps = args.warmup + args.steps
    plans = []
    for _ in range(steps):  # every member exchanges with one partner; batches keep both directions
        perm = rng.permutation(n).astype(np.uint32).reshape(-1, 2)
        batches = []
        for i in range(0, len(perm), BATCH // 2):
            m = perm[i:i + BATCH // 2]
            p = np.zeros(2 * len(m), PP_PAIR_DTYPE)
            p["receiver"] = np.concatenate([m[:, 0], m[:, 1]])
            p["sender"] = np.concatenate([m[:, 1], m[:, 0]])
            batches.append(torch.from_numpy(p.view(np.uint64).copy()).cuda())
        plans.append(batches)
    torch.cuda.synchronize()
    evs = []

    def step(i, timed):
        for b in plans[i]:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            eng.push_pull_device(b.data_ptr(), b.numel())
            e1.record(stream)
            if timed:
                evs.append((e0, e1, b.numel()))

    for i in range(args.warmup):
        step(i, False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.warmup, steps):
        step(i, True)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ms = [a.elapsed_time(b) for a, b, _ in evs]
    pairs_per_launch = float(np.mean([k for _, _, k in evs]))
    avg_ms = float(np.mean(ms))
    sb = state_bytes(cfg)
    # algorithmic bytes per pair: the sender's local_state read once + the receiver's view
    # and event-buffer rows read (writes are the few changed entries)
    per_pair = sb + cfg.n_subjects * 16 + cfg.event_buffer_size * (12 + 8 * cfg.slot_k)
    achieved = per_pair * pairs_per_launch / (avg_ms / 1e3) / 1e9
    eng.close()
    merges = n * args.steps
    return {
        "metric": "push/pull merges/s", "value": merges / wall, "unit": "merge_remote_state/s",
        "ms_per_step": wall / args.steps * 1e3, "dtype": "u64",
        "config": {"workload": f"push/pull anti-entropy: {n} members each exchange local_state with one random "
                               f"partner (matching, both directions), {SUBJECTS} tracked subjects, event buffer "
                               f"{cfg.event_buffer_size}, state from {SETTLE_ROUNDS} settled configs[1] rounds + "
                               f"256 user events/round",
                   "members": n, "members_per_gpu": n, "pairs_per_launch": pairs_per_launch,
                   "parallelism": "single GPU"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": "pp_snapshot+pp_merge_kernel",
                     "bytes_per_unit": per_pair, "units_per_launch": pairs_per_launch,
                     "bytes_per_launch": per_pair * pairs_per_launch, "avg_launch_ms": avg_ms},
        "scaling": "weak",
    }


def cpu_baseline_pushpull(args, seconds_target=10.0):
    import ctypes as C
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import gossip_harness as H  # test infrastructure: checker / CPU baseline only
    from ruserf_amd import workload as W
    from ruserf_amd.gossip import PP_PAIR_DTYPE
    n = 50_000
    cfg = pp_cfg(n, SETTLE_ROUNDS)
    subj, acts, ml = workload(n, SETTLE_ROUNDS)
    w = H.oracle_world(cfg, subj, W.initial_views(SUBJECTS))
    for t in range(SETTLE_ROUNDS):
        H.oracle_round(w, t, ml[t], acts[t])
    rng = np.random.Generator(np.random.Philox(SEED + 3))
    done, spent = 0, 0.0
    while spent < seconds_target:
        m = rng.permutation(n).astype(np.uint32)[:4096].reshape(-1, 2)
        p = np.zeros(2 * len(m), PP_PAIR_DTYPE)
        p["receiver"] = np.concatenate([m[:, 0], m[:, 1]])
        p["sender"] = np.concatenate([m[:, 1], m[:, 0]])
        t0 = time.perf_counter()
        H.oracle_push_pull(w, p)
        spent += time.perf_counter() - t0
        done += len(p)
    H.L.orc_world_free(C.byref(w))
    return {"value": done / spent, "unit": "merge_remote_state/s", "cores": 1, "kind": "port",
            "sample": f"oracle push/pull, {n} members settled, {done} merges ({spent:.1f}s), single thread"}
