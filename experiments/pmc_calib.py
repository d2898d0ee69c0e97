"""Reads the pmc_calib rocprofv3 CSVs (trace, FETCH_SIZE, WRITE_SIZE passes) and prints,
per access shape, true bytes, counter bytes, ratio and achieved GB/s."""
import csv, sys, collections

d = sys.argv[1]
names = [l.split()[1:3] for l in open(f"{d}/calib.log") if l.startswith("calib ") and "done" not in l]
def rows(p, counter=None):
    out = []
    for r in csv.DictReader(open(p)):
        if "rocclr" in r["Kernel_Name"]:
            continue
        if counter and r["Counter_Name"] != counter:
            continue
        out.append(r)
    return out
tr = rows(f"{d}/trace/run_kernel_trace.csv")
fe = rows(f"{d}/fetch/run_counter_collection.csv", "FETCH_SIZE")
wr = rows(f"{d}/write/run_counter_collection.csv", "WRITE_SIZE")
print(f"{'shape':16} {'true MB':>9} {'FETCH MB':>9} {'ratio':>6} {'WRITE MB':>9} {'ratio':>6} {'GB/s':>7}")
for i, (nm, b) in enumerate(names):
    b = int(b)
    t = (int(tr[i]["End_Timestamp"]) - int(tr[i]["Start_Timestamp"])) / 1e9
    f = float(fe[i]["Counter_Value"]) * 1024
    w = float(wr[i]["Counter_Value"]) * 1024
    print(f"{nm:16} {b/1e6:9.1f} {f/1e6:9.1f} {f/b:6.3f} {w/1e6:9.1f} {w/b:6.3f} {b/t/1e9:7.0f}")
