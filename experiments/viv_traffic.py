"""Per-ablation-variant FETCH_SIZE / WRITE_SIZE averages of vivaldi_observe_kernel
(from viv_traffic.sh) and the corrected HBM traffic of the full kernel:
  streamed reads are tallied at 1/2 (experiments/pmc_calib: stream_read* ratio 0.500),
  random 96-B row gathers at 1.0 of the useful bytes (gather96 ratio 0.998),
  writes at 1.0 (stream_write* 1.000)."""
import csv, collections, json, re, sys

d = sys.argv[1]
def per_variant(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or "vivaldi_observe_kernel" not in r["Kernel_Name"]:
            continue
        m = re.search(r"vivaldi_observe_kernel<8, 3, 20, (\d+)", r["Kernel_Name"])
        agg[int(m.group(1))].append(float(r["Counter_Value"]) * 1024)
    return {k: sum(v) / len(v) for k, v in agg.items()}
f = per_variant(f"{d}/fetch/run_counter_collection.csv", "FETCH_SIZE")
w = per_variant(f"{d}/write/run_counter_collection.csv", "WRITE_SIZE")
t = json.load(open(f"{d}/times.json"))
names = {0: "full", 1: "no_peer_gather", 2: "no_filter", 4: "no_window", 8: "no_self_row_read", 16: "no_row_write",
         32: "no_probe_inputs", 7: "self_row_only", 63: "compute_only"}
for k in sorted(f):
    print(f"mask {k:2d} {names[k]:17} FETCH {f[k]/1e9:7.3f} GB  WRITE {w.get(k, 0)/1e9:7.3f} GB  {t.get(names[k], 0):7.3f} ms")
gather_cnt = f[0] - f[1]
stream_cnt = f[1]
traffic = 2 * stream_cnt + gather_cnt + w[0]
print(json.dumps({"fetch_counter": f[0], "write_counter": w[0], "gather_counter": gather_cnt,
                  "stream_counter": stream_cnt, "traffic_bytes": traffic, "ms_full": t["full"]}))
