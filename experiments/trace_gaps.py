"""Per-round span vs kernel-busy time from a rocprofv3 kernel trace (the last 5 rounds, delimited
by the round's last kernel NAME), and the idle gaps between consecutive launches by the pair of
kernels around them.  Usage: trace_gaps.py run_kernel_trace.csv merge_kernel"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
key = sys.argv[2]
ends = [i for i, r in enumerate(rows) if key in r["Kernel_Name"] and "big" not in r["Kernel_Name"]]
a, b = ends[-6] + 1, ends[-1]
seg = rows[a:b + 1]
t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
n = 5
print(f"per round: span {(t1 - t0) / 1e6 / n:.3f} ms, kernel busy {busy / 1e6 / n:.3f} ms, launches {len(seg) / n:.1f}")
gaps = collections.Counter()
cnt = collections.Counter()
for p, q in zip(seg, seg[1:]):
    g = int(q["Start_Timestamp"]) - int(p["End_Timestamp"])
    k = (p["Kernel_Name"].split("(")[0][-40:], q["Kernel_Name"].split("(")[0][-40:])
    gaps[k] += g
    cnt[k] += 1
tot = sum(gaps.values())
print(f"gaps: {tot / 1e3 / n:.1f} us per round")
for k, v in gaps.most_common(15):
    print(f"  {v / 1e3 / n:7.1f} us/round  x{cnt[k] / n:.1f}  {k[0]} -> {k[1]}")
