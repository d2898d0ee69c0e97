"""Per-kernel mean duration over the last N rounds of a rocprofv3 kernel trace (rounds are
delimited by merge_kernel launches).  Usage: trace_last.py kernel_trace.csv [N]"""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
merges = [i for i, r in enumerate(rows) if "merge_kernel<" in r["Kernel_Name"]]
start = merges[-n - 1] + 1 if len(merges) > n else 0
tot = collections.defaultdict(float)
for r in rows[start:merges[-1] + 1]:
    m = re.search(r"::(\w+<[^>]*>|\w+)\(", r["Kernel_Name"])
    k = m.group(1) if m else r["Kernel_Name"][:50]
    tot[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
span = (int(rows[merges[-1]]["End_Timestamp"]) - int(rows[start]["Start_Timestamp"])) / 1e3
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"{v / n:9.1f} us/round  {k}")
print(f"{sum(tot.values()) / n:9.1f} us/round  kernels total; span {span / n:.1f} us/round")
