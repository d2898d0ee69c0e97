"""Per-kernel time over the last K rounds of two rocprofv3 kernel traces (e.g. the bucket path on
one rank against the single context).  A round ends at its merge kernel; the window is the K
rounds before the last merge.  Usage: trace_compare.py A.csv B.csv [K]"""
import csv
import sys
from collections import defaultdict


def window(path, k):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    merges = [i for i, r in enumerate(rows) if "merge_kernel" in r["Kernel_Name"] and "big" not in r["Kernel_Name"]]
    lo, hi = merges[-k - 1] + 1, merges[-1]
    acc = defaultdict(float)
    for r in rows[lo:hi + 1]:
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]
        acc[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 / k
    span = (int(rows[hi]["End_Timestamp"]) - int(rows[lo]["Start_Timestamp"])) / 1e3 / k
    return acc, span


def main():
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    a, sa = window(sys.argv[1], k)
    b, sb = window(sys.argv[2], k)
    print(f"{'kernel':62s} {'A us/round':>11s} {'B us/round':>11s} {'A-B':>8s}")
    for n in sorted(set(a) | set(b), key=lambda n: -(a.get(n, 0) + b.get(n, 0))):
        print(f"{n:62s} {a.get(n, 0):11.1f} {b.get(n, 0):11.1f} {a.get(n, 0) - b.get(n, 0):8.1f}")
    print(f"{'round span':62s} {sa:11.1f} {sb:11.1f} {sa - sb:8.1f}")


if __name__ == "__main__":
    main()
