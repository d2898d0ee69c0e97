#!/usr/bin/env python3
"""bench.py — the driver's benchmark contract for ruserf_amd.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload gossip|vivaldi|pushpull|churn]

BASELINE.json's metric has two halves, "gossip node-rounds/sec (whole node) at 16M
members; Vivaldi updates/sec".  The default run measures both in one invocation: the
gossip leg is the line's `value`, the Vivaldi leg (configs[4], 64M members) is the
line's `vivaldi` object with its own ms_per_step, roofline and cpu_baseline.

One step = one pass of the hot path over one batch of synthetic input:
  gossip  : one gossip round over the shard's members -> metric "node-rounds/s".
            Default 1M members per GPU (BASELINE configs[1] at N=1) in the reference's
            queue regime: the intent queue DEFAULT_QUEUE_DEPTH (8 704) deep, each member's
            QueueChecker pruning it to 4 096 every 150 rounds on its own phase inside the
            timed rounds.  configs[2]'s 2M-per-GPU shard is `--members 2000000`; the line
            also carries labelled points at 2M (the same regime) and with bounded 64-slot
            queues (model points).
  vivaldi : one Vivaldi round (every member probes one neighbour and runs
            CoordinateClient::update) (configs[4]) -> "Vivaldi updates/s"
Multi-GPU: one process per GPU (torch.distributed over RCCL), members sharded
by contiguous id range, weak scaling.  Rank 0 prints ONE JSON line.
"""
import argparse
import ctypes as C
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

SEED = 0x5EED5EED
# algorithmic HBM bytes per Vivaldi update in rsf_vivaldi_observe:
# reads self 88 + peer 88 + adjustment window 160 + window index 4 + filter samples 24 + filter meta 4
#       + probe input (peer id 4 + rtt ns 8),
# writes self 88 + window slot 8 + window index 4 + filter sample 8 + filter meta 4  (D=8, W=20, F=3)
VIVALDI_BYTES = 492
HBM_PEAK_GBS = 8000.0
# the gossip headline runs the reference's queue regime: the intent queue deep enough that
# nothing is dropped between QueueChecker ticks (4096 after a tick + ~24 a round x 150 rounds)
DEFAULT_QUEUE_DEPTH = 8704


class CudaArray:
    """Zero-copy view of engine-owned HBM as a torch tensor (for collectives)."""

    def __init__(self, ptr, shape, typestr):
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": typestr, "data": (int(ptr), False),
                                         "version": 3, "strides": None}


def env_rank():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def cpu_info():
    model = platform.processor() or "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model


def cpu_threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", n))))


def barrier(world):
    if world > 1:
        torch.distributed.barrier()


def coll_device():
    """Tensors for the bench's own small collectives: HBM under RCCL, host under gloo."""
    return "cpu" if torch.distributed.get_backend() == "gloo" else "cuda"


def max_over_ranks(x, world):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=coll_device())
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, world):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=coll_device())
    torch.distributed.all_reduce(t)
    return float(t.item())


# --------------------------------------------------------------------------- vivaldi
def run_vivaldi(args, rank, world):
    from ruserf_amd import CoordinateClients, CoordinateOptions
    per = args.members // world if args.members_total else args.members
    n = per * world
    lo, hi = rank * per, (rank + 1) * per
    stream = torch.cuda.current_stream()  # a non-default stream (set in main)
    g = CoordinateClients(n, 16, CoordinateOptions(), seed=SEED, device=torch.cuda.current_device(),
                          shard=(lo, hi))
    g.set_stream(stream.cuda_stream)
    table = None

    R = max(1, args.refresh_every)
    # N > 1, R = 1: the targeted exchange (only the rows of this round's remote peers,
    # fetched from their owners before the round); R > 1 or --vivaldi-exchange allgather:
    # an all-gather of the table after every R-th round
    targeted = world > 1 and R == 1 and args.vivaldi_exchange == "targeted"
    sv = None
    if targeted:
        from ruserf_amd.dist import ShardedVivaldi
        sv = ShardedVivaldi(g, rank, world)
        sv.time_chunks = True

    refresher = None
    if world > 1 and not targeted:
        from ruserf_amd.dist import VivaldiTableRefresh
        refresher = VivaldiTableRefresh(g, rank, world, R)

    def refresh(r):
        if refresher is not None:
            refresher.after_round(r, read_ptr[0])

    # the probe inputs (peer id, observed rtt) of every round are generated up front by
    # the synthetic network and are resident in HBM when the timed region starts
    rounds = args.warmup + args.steps
    peer = torch.empty((rounds, per), dtype=torch.int32, device="cuda")
    rtt = torch.empty((rounds, per), dtype=torch.int64, device="cuda")
    for r in range(rounds):
        g.gen_probes(r, peer[r].data_ptr(), rtt[r].data_ptr())
    step = [0]

    read_ptr = [None]  # the table a round reads (the other one after it)

    chunks = max(1, getattr(args, "vivaldi_chunks", 1)) if targeted else 1

    def observe(r):
        read_ptr[0] = g.table_ptr()[0]
        if chunks > 1:  # the exchange of chunk i + 1 beside the observe of chunk i (round_chunked)
            sv.round_chunked(r, peer[r].data_ptr(), rtt[r].data_ptr(), chunks=chunks)
        else:
            g.observe(r % 16, peer[r].data_ptr(), rtt[r].data_ptr(), None, r)

    def fetch(r):
        if targeted and chunks == 1:
            sv.fetch(peer[r].data_ptr())

    def presend(r):
        # round r + 1's requests go out while round r's observe runs
        if targeted and chunks == 1 and r + 1 < rounds:
            sv.presend(peer[r + 1].data_ptr())

    for _ in range(args.warmup):
        fetch(step[0])
        observe(step[0])
        presend(step[0])
        refresh(step[0])
        step[0] += 1
    torch.cuda.synchronize()
    barrier(world)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kernel_ms = []
    for i in range(args.steps):
        fetch(step[0])
        evs[i][0].record(stream)
        observe(step[0])
        evs[i][1].record(stream)
        presend(step[0])
        refresh(step[0])
        step[0] += 1
    torch.cuda.synchronize()
    barrier(world)
    wall = time.perf_counter() - t0
    kernel_ms = [a.elapsed_time(b) for a, b in evs]
    if chunks > 1:  # the observe kernels' own time: the chunks' launches summed per round
        kernel_ms = [sum(a.elapsed_time(b) for a, b in rnd) for rnd in sv.chunk_events[-args.steps:]]
    wall = max_over_ranks(wall, world)
    if targeted and not sv.check():
        raise RuntimeError("vivaldi exchange: a request bucket overflowed")
    avg_kernel_s = float(np.mean(kernel_ms)) / 1e3
    updates = per * world * args.steps
    value = updates / wall
    achieved = VIVALDI_BYTES * per / avg_kernel_s / 1e9
    g.close()
    return {
        "metric": "Vivaldi updates/s", "value": value, "unit": "updates/s",
        "ms_per_step": wall / args.steps * 1e3, "dtype": "f64",
        "config": {"workload": f"Vivaldi rounds (BASELINE configs[4] shape), {n} members, D=8 f64, height + "
                               f"latency filter F=3, adjustment window W=20, 16 neighbours/member probed round-robin, "
                               f"probe inputs (peer, rtt) pre-generated in HBM",
                   "members": n, "members_per_gpu": per, "parallelism": f"members sharded x{world}",
                   "table_refresh_every_rounds": R,
                   "exchange": ((f"targeted peer rows, the round pipelined in {chunks} member chunks" if chunks > 1
                                 else "targeted peer rows") if targeted else f"table all-gather every {R} rounds")
                   if world > 1 else None},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": "vivaldi_observe_pipe_kernel<3>", "bytes_per_unit": VIVALDI_BYTES,
                     "units_per_launch": per, "bytes_per_launch": VIVALDI_BYTES * per,
                     "avg_launch_ms": avg_kernel_s * 1e3},
        # --members is per GPU unless --members-total; the default keeps 64M members in total
        "scaling": "strong" if args.members_total else "weak",
    }


def cpu_baseline_vivaldi(seconds_target=8.0):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O  # test infrastructure: the checker / CPU baseline only
    L = O.lib()
    th = cpu_threads()
    n = 2_000_000
    p = O.VivaldiPop()
    oo = O.default_opts()
    L.orc_vivaldi_pop_init(C.byref(p), n, 16, C.byref(oo), SEED)
    L.orc_vivaldi_pop_rounds(C.byref(p), 0, 1, th)  # warm (page faults)
    rounds, t_total, r = 0, 0.0, 1
    while t_total < seconds_target and rounds < 200:
        t = time.perf_counter()
        L.orc_vivaldi_pop_rounds(C.byref(p), r, 1, th)
        t_total += time.perf_counter() - t
        rounds += 1
        r += 1
    L.orc_vivaldi_pop_free(C.byref(p))
    return {"value": n * rounds / t_total, "unit": "updates/s", "cores": th, "kind": "port",
            "sample": f"oracle Vivaldi rounds, {n} members x {rounds} rounds ({t_total:.1f}s) on {th} threads, "
                      f"{cpu_info()}"}


def model_point(args, rank, world, members):
    """One more gossip measurement with the bounded 64-slot queues (see main)."""
    from bench_gossip import run_gossip
    a = argparse.Namespace(**vars(args))
    a.members, a.queue_cap, a.settle = members, 64, None
    a.queue_depth, a.check_every = 0, 0
    torch.cuda.empty_cache()
    r = run_gossip(a, rank, world)
    keep = ["value", "unit", "ms_per_step", "merges_per_s", "records_per_round_per_gpu", "queue_pruned_per_round",
            "queue_pruned_per_merged_record", "error_members", "cub_canaries_intact", "phases_ms_per_round"]
    out = {"metric": r["metric"], "steps": args.steps, "warmup": args.warmup, **{k: r[k] for k in keep},
           "config": r["config"],
           "what": "model point: queues bounded at 64 slots, pruned on insert (the reference's queues are "
                   "unbounded between QueueChecker ticks); not the reference's regime"}
    out["roofline"] = {k: r["roofline"][k] for k in ["bound", "achieved", "peak", "unit", "frac", "kernel",
                                                      "bytes_per_launch", "avg_launch_ms"]}
    return out


def regime_point(args, rank, world, members):
    """configs[2]'s per-GPU shard (2M members) in the same reference queue regime as the line,
    same box, same call: a labelled point beside the configs[1] headline."""
    from bench_gossip import run_gossip
    a = argparse.Namespace(**vars(args))
    a.members = members
    torch.cuda.empty_cache()
    r = run_gossip(a, rank, world)
    keep = ["value", "unit", "ms_per_step", "merges_per_s", "records_per_round_per_gpu", "queue_pruned_per_round",
            "error_members", "cub_canaries_intact", "phases_ms_per_round", "queue_regime",
            "deep_path_members_per_round"]
    out = {"metric": r["metric"], "steps": args.steps, "warmup": args.warmup, **{k: r[k] for k in keep},
           "config": r["config"],
           "what": "BASELINE configs[2]'s per-GPU shard (2M members; 16M over 8 GPUs) in the reference's queue "
                   "regime, one GPU (the multi-GPU exchange is not in this point)"}
    out["roofline"] = {k: r["roofline"][k] for k in ["bound", "achieved", "peak", "unit", "frac", "kernel",
                                                      "bytes_per_launch", "avg_launch_ms"]}
    return out


def c1_leg(rounds=1000, n=1000, with_gpu=True):
    """BASELINE configs[0] / SURVEY §8(d) C1: Vivaldi over a 1k-node synthetic RTT matrix on
    the CPU path -- the oracle (the C restatement of CoordinateClient::update; the Rust
    reference cannot be built here) on one thread: n clients, each probing one of its 16
    fixed neighbours per round (peer coordinates from the previous round), `rounds` rounds
    = n x rounds updates.  Reports updates/s and the final median |est - true| / true over
    all pairs.  with_gpu: the same rounds on the HIP engine, bit-exact against it."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O  # test infrastructure: the C1 CPU path and its checker
    L = O.lib()
    p = O.VivaldiPop()
    oo = O.default_opts()
    L.orc_vivaldi_pop_init(C.byref(p), n, 16, C.byref(oo), SEED)
    t = time.perf_counter()
    L.orc_vivaldi_pop_rounds(C.byref(p), 0, rounds, 1)
    spent = time.perf_counter() - t
    med = L.orc_vivaldi_pop_median_rel_error(C.byref(p))
    out = {"config": f"BASELINE configs[0]: {n} Vivaldi clients, D=8, default CoordinateOptions, 16 neighbours "
                     f"each probed one per round with x(1+U[0,0.1)) jitter, {rounds} rounds = {n * rounds} updates",
           "cpu_updates_per_s": n * rounds / spent, "cpu_seconds": spent, "cores": 1, "kind": "port",
           "cpu_model": cpu_info(), "median_rel_rtt_error_all_pairs": med, "resets": int(p.resets)}
    if with_gpu:
        from ruserf_amd import CoordinateClients, CoordinateOptions
        g = CoordinateClients(n, 16, CoordinateOptions(), seed=SEED, device=torch.cuda.current_device())
        g.set_stream(torch.cuda.current_stream().cuda_stream)
        for r in range(rounds):
            g.round(r)
        torch.cuda.synchronize()
        exp = O.arr(p.rows_cur, n * p.row_stride, np.float64).reshape(n, p.row_stride)
        out["gpu_bit_exact"] = bool(np.array_equal(g.get_rows().view(np.uint64), exp.view(np.uint64)))
        g.close()
    L.orc_vivaldi_pop_free(C.byref(p))
    return out


# --------------------------------------------------------------------------- traffic
def attach_traffic(workload, res):
    """roofline.traffic = HBM bytes per launch of the dominant kernel from the rocprofv3
    PMC passes committed under profiles/ (scripts/make_traffic.py; corrections in
    DESIGN.md §Measurement), when this run's kernel and size match the profiled one."""
    rl = res["roofline"]
    try:
        with open(os.path.join(ROOT, "profiles", "traffic.json")) as f:
            ent = json.load(f).get(workload)
    except (OSError, ValueError):
        ent = None
    if not ent or ent["kernel"] != rl["kernel"] or ent["members_per_gpu"] != res["config"]["members_per_gpu"]:
        return
    rl["traffic"] = ent["traffic_bytes_per_launch"]
    rl["traffic_unit"] = "bytes/launch"
    rl["traffic_vs_algorithmic"] = ent["traffic_bytes_per_launch"] / rl["bytes_per_launch"]
    rl["traffic_source"] = ent["source"]
    # the dominant kernel against the floor of its access pattern (random 64-B sectors read
    # and written), measured by a microbenchmark with no protocol logic
    try:
        with open(os.path.join(ROOT, "profiles", "pattern_floor.json")) as f:
            fl = json.load(f).get(workload)
    except (OSError, ValueError):
        fl = None
    if fl and fl["kernel"] == rl["kernel"] and fl["members_per_gpu"] == res["config"]["members_per_gpu"]:
        rl["pattern_floor"] = {"ms": fl["floor_ms"], "kernel_ms": rl["avg_launch_ms"],
                               "floor_over_kernel": fl["floor_ms"] / rl["avg_launch_ms"], "what": fl["what"],
                               "source": fl["source"]}


# --------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["gossip", "vivaldi", "pushpull", "churn"], default=None)
    ap.add_argument("--members", type=int, default=None, help="members per GPU")
    ap.add_argument("--members-total", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--queue-cap", type=int, default=64,
                    help="gossip: slots per transmit-limited queue (1..256; the reference's max_queue_depth is 4096)")
    ap.add_argument("--queue-depth", type=int, default=None,
                    help="gossip: intent queue depth above --queue-cap (<= 64): a register head plus an HBM tail, "
                         "pruned only by the QueueChecker every --check-every rounds (the reference's regime; default "
                         "8704: max_queue_depth 4096 plus what 150 rounds add between ticks, with margin); 0: the "
                         "bounded --queue-cap model")
    ap.add_argument("--check-every", type=int, default=None,
                    help="gossip: a QueueChecker tick (prune to max_queue_depth 4096) every K rounds inside the round "
                         "loop, the timed window ending with one (default: 150 with --queue-depth, else none)")
    ap.add_argument("--no-extra-points", action="store_true",
                    help="gossip: skip the configs[1] points (1M members, 64- and 256-slot queues)")
    ap.add_argument("--settle", type=int, default=None,
                    help="gossip: untimed rounds before warmup (default 330 in the queue regime: queues at their "
                         "steady state past two checker ticks; 12 with bounded queues: saturated)")
    ap.add_argument("--no-vivaldi", action="store_true", help="gossip: skip the Vivaldi leg of the line")
    ap.add_argument("--ring-rounds", type=int, default=None,
                    help="gossip: rounds of rumor blocks the rumor ring holds per generation (default: the whole "
                         "run in the queue regime, so nothing expires)")
    ap.add_argument("--refresh-every", type=int, default=1,
                    help="vivaldi, N>1: all-gather the coordinate table after every R-th round (C5: 1 and 8)")
    ap.add_argument("--vivaldi-exchange", choices=["targeted", "allgather"], default="targeted",
                    help="vivaldi, N>1, R=1: fetch only the round's remote peer rows, or all-gather the table")
    ap.add_argument("--vivaldi-chunks", type=int, default=4,
                    help="vivaldi, N>1, targeted: the round pipelined in this many member chunks (chunk i observed "
                         "while chunk i+1's rows are exchanged); 1: the exchange before the whole observe")
    args = ap.parse_args()
    if args.queue_depth is None:
        args.queue_depth = DEFAULT_QUEUE_DEPTH if args.queue_cap <= 64 else 0
    if args.check_every is None:
        args.check_every = 150 if args.queue_depth else 0
    rank, world, local = env_rank()
    if world != args.gpus and world == 1 and args.gpus > 1:
        print("run multi-GPU through torch.distributed.run (one process per GPU)", file=sys.stderr)
        sys.exit(2)
    # RSF_DIST_BACKEND=gloo rehearses the multi-rank path on fewer GPUs than ranks (ranks
    # share devices, the exchange is host-staged); the driver's runs use RCCL ("nccl")
    backend = os.environ.get("RSF_DIST_BACKEND", "nccl")
    dev = local % torch.cuda.device_count() if backend == "gloo" else local
    torch.cuda.set_device(dev)
    # every engine launch goes to this stream; torch's default stream handle is NULL,
    # which the C ABI would read as "the context's own stream"
    torch.cuda.set_stream(torch.cuda.Stream())
    # RSF_FORCE_SHARDED=1 (under torch.distributed.run, one rank): the gossip bench runs the
    # multi-GPU code path (ShardedGossip, RCCL collectives) on one GPU, to price its overhead
    forced = os.environ.get("RSF_FORCE_SHARDED") == "1"
    if world > 1 or forced:
        if backend == "gloo":
            torch.distributed.init_process_group("gloo")
        else:
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", dev))
    import ruserf_amd
    try:
        from ruserf_amd import gossip  # noqa: F401
        have_gossip = True
    except ImportError:
        have_gossip = False
    workload = args.workload or ("gossip" if have_gossip else "vivaldi")
    if workload == "vivaldi":
        if args.members is None:  # BASELINE configs[4]: 64M members in total, sharded
            args.members, args.members_total = 64_000_000, True
        res = run_vivaldi(args, rank, world)
        cpu = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline_vivaldi()
            res["configs0_c1"] = c1_leg()
    elif workload == "churn":
        from bench_churn import cpu_baseline_churn, run_churn
        res = run_churn(args, rank, world)
        cpu = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline_churn(args)
    elif workload == "pushpull":
        from bench_pushpull import cpu_baseline_pushpull, run_pushpull
        args.members = args.members or 1_000_000
        res = run_pushpull(args, rank, world)
        cpu = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline_pushpull(args)
    else:
        from bench_gossip import run_gossip, cpu_baseline_gossip, cpu_baseline_gossip_deep
        # BASELINE configs[1] (1M members on one MI355X; configs[2]'s 16M do not fit one GPU)
        # in the reference's queue regime; per GPU under torch.distributed (weak scaling)
        args.members = args.members or 1_000_000
        res = run_gossip(args, rank, world)
        cpu = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline_gossip_deep(args) if args.queue_depth else cpu_baseline_gossip(args)
        attach_traffic(workload, res)
        if world == 1 and not args.no_extra_points:
            # labelled model points, same box, same call: the bounded 64-slot queue (prunes on
            # insert, which the reference never does) at configs[1] and at configs[2]'s 2M shard
            if args.queue_depth and args.members == 1_000_000:
                res["configs2_shard_regime"] = regime_point(args, rank, world, 2_000_000)
            pts = [model_point(args, rank, world, 1_000_000), model_point(args, rank, world, 2_000_000)]
            e64 = pts[0]["phases_ms_per_round"].get("emit_kernel")
            edeep = res["phases_ms_per_round"].get("emit_kernel")
            if res.get("queue_regime") and e64 and edeep:
                res["queue_regime"]["emit_ms_vs_q64_same_call"] = edeep / e64
            res["model_points_q64"] = pts
        if not args.no_vivaldi:
            # the metric's second half, timed in the same invocation (configs[4]: 64M members)
            vargs = argparse.Namespace(**vars(args))
            vargs.members, vargs.members_total = 64_000_000, True
            torch.cuda.empty_cache()
            vres = run_vivaldi(vargs, rank, world)
            attach_traffic("vivaldi", vres)
            vcpu = None
            if rank == 0 and world == 1 and not args.no_cpu_baseline:
                vcpu = cpu_baseline_vivaldi()
            res["vivaldi"] = {"metric": vres["metric"], "value": vres["value"], "unit": vres["unit"],
                              "steps": args.steps, "warmup": args.warmup, "ms_per_step": vres["ms_per_step"],
                              "scaling": vres["scaling"], "dtype": vres["dtype"], "config": vres["config"],
                              "roofline": vres["roofline"], "cpu_baseline": vcpu}
            if rank == 0 and world == 1 and not args.no_cpu_baseline:
                res["vivaldi"]["configs0_c1"] = c1_leg()
    if workload != "gossip":
        attach_traffic(workload, res)
    if rank == 0:
        line = {
            "metric": res["metric"], "value": res["value"], "unit": res["unit"], "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": res["ms_per_step"],
            "higher_is_better": True, "scaling": res.get("scaling", "weak"), "vs_baseline": None, "dtype": res["dtype"],
            "data": "synthetic", "config": res["config"], "roofline": res["roofline"], "cpu_baseline": cpu,
        }
        for k in res:
            if k not in line and k not in ("metric",):
                line[k] = res[k]
        print(json.dumps(line), flush=True)
    if world > 1 or forced:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
