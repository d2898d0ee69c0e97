#!/usr/bin/env python3
"""Turns the rocprofv3 outputs of scripts/profile.sh (gpurun_out/prof_<tag>_{trace,fetch,write})
into committed summaries under profiles/<round>/:

  <tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary, verbatim
  <tag>_summary.md         per-kernel average duration over the TIMED dispatches (the last
                           --steps launches), FETCH_SIZE / WRITE_SIZE per launch, the bench
                           line printed under the profiler

Usage: summarize_profile.py ROUND TAG STEPS [TAG STEPS ...]
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def per_dispatch(path, counter=None):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if counter and r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        if counter:
            d[name].append(float(r["Counter_Value"]) * 1024)  # rocprofv3 reports KiB
        else:
            d[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return d


def bench_line(log):
    for line in open(log):
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    return None


def summarize(rnd, tag, steps):
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    base = os.path.join(OUT, f"prof_{tag}")
    shutil.copy(f"{base}_trace/run_kernel_stats.csv", os.path.join(dst, f"{tag}_kernel_stats.csv"))
    dur = per_dispatch(f"{base}_trace/run_kernel_trace.csv")
    fetch = per_dispatch(f"{base}_fetch/run_counter_collection.csv", "FETCH_SIZE")
    write = per_dispatch(f"{base}_write/run_counter_collection.csv", "WRITE_SIZE")
    line = bench_line(f"{base}_trace.log")
    rows = []
    for name, v in dur.items():
        if len(v) < steps:
            continue
        t = v[-steps:]
        f = fetch.get(name, [])[-steps:]
        w = write.get(name, [])[-steps:]
        rows.append((sum(t) / steps, name, len(v), sum(f) / max(1, len(f)), sum(w) / max(1, len(w))))
    rows.sort(reverse=True)
    with open(os.path.join(dst, f"{tag}_summary.md"), "w") as fo:
        fo.write(f"# rocprofv3 summary: {tag}\n\n")
        fo.write("Source: `scripts/profile.sh` (one `--kernel-trace --stats` pass, then separate `--pmc FETCH_SIZE` "
                 "and `--pmc WRITE_SIZE` passes of the same command).  Averages are over the last "
                 f"{steps} dispatches of each kernel (the bench's timed steps).  FETCH_SIZE/WRITE_SIZE are the "
                 "raw counters (KiB x 1024) per launch, uncorrected: see DESIGN.md §Measurement for the gfx950 "
                 "corrections (`experiments/pmc_calib`).\n\n")
        fo.write("| kernel | dispatches | avg ms (timed) | FETCH_SIZE MB/launch | WRITE_SIZE MB/launch |\n")
        fo.write("|---|---|---|---|---|\n")
        for t, name, cnt, f, w in rows:
            short = name if len(name) < 90 else name[:87] + "..."
            fo.write(f"| `{short}` | {cnt} | {t:.3f} | {f / 1e6:.1f} | {w / 1e6:.1f} |\n")
        if line:
            fo.write("\nBench line printed under the profiler (trace pass):\n\n```json\n")
            fo.write(json.dumps(line) + "\n```\n")
    print(f"wrote profiles/{rnd}/{tag}_summary.md")
    return rows


if __name__ == "__main__":
    rnd = sys.argv[1]
    args = sys.argv[2:]
    for i in range(0, len(args), 2):
        summarize(rnd, args[i], int(args[i + 1]))
