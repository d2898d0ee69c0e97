#!/usr/bin/env python3
"""Writes profiles/traffic.json: corrected HBM bytes per launch of each bench's dominant
kernel, from the PMC passes under gpurun_out/ (see DESIGN.md §Measurement).

gfx950 corrections (measured by experiments/pmc_calib, profiles/r01/pmc_calibration.txt):
  * coalesced streaming reads are tallied at 1/2 by FETCH_SIZE (4/8/16 B per lane alike);
  * random gathers of <= 64 B count one 64-B sector each, i.e. the HBM bytes they move;
  * WRITE_SIZE is exact for streaming stores.
Vivaldi (vivaldi_observe_pipe_kernel): the peer-row gather (96 B per member, tallied at
0.998, gather96) is modelled and the rest of FETCH is the coalesced streams (tallied at 1/2,
non-temporal loads alike: stream_read*_nt); byte-wide loads (the u8 window index) are not
tallied at all (stream_read1), so they are added from the model:
    traffic = 2*(FETCH - 0.998*gather) + gather + idx + WRITE   (idx = 1 B per member).
The modelled FETCH (streams/2 + 0.998*gather) is printed beside the measured one.
Gossip (merge_kernel): the streamed bytes are modelled (the (sender, peer) groups' record
slots, cap_t x 8 B + a 4-B count each) and corrected (x2); the rest of FETCH is gather:
traffic = FETCH + stream/2 + WRITE."""
import csv
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
RND = sys.argv[1] if len(sys.argv) > 1 else "r01"


def last(path, counter, pat, k=5):
    v = [float(r["Counter_Value"]) * 1024 for r in csv.DictReader(open(path))
         if r["Counter_Name"] == counter and pat in r["Kernel_Name"]]
    return sum(v[-k:]) / len(v[-k:])


# entries whose profile is not under gpurun_out/ now are kept from the committed file
try:
    res = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))
except (OSError, ValueError):
    res = {}
VTAG = os.environ.get("VIV_TAG", "viv_r01c")
v = os.path.join(OUT, f"prof_{VTAG}")
if os.path.isdir(f"{v}_fetch"):
    f_viv = last(f"{v}_fetch/run_counter_collection.csv", "FETCH_SIZE", "vivaldi_observe_pipe_kernel")
    w_viv = last(f"{v}_write/run_counter_collection.csv", "WRITE_SIZE", "vivaldi_observe_pipe_kernel")
    vline = next(json.loads(x) for x in open(f"{v}_trace.log") if x.startswith("{") and '"metric"' in x)
    nv = vline["config"]["members_per_gpu"]
    gather = 96 * nv
    streams = nv * (96 + 16 + 160 + 4 + 8)  # own row, filter record, window, peer id, rtt (all coalesced)
    traffic_v = 2 * (f_viv - 0.998 * gather) + gather + nv + w_viv
    res["vivaldi"] = {"kernel": "vivaldi_observe_pipe_kernel<3>", "members_per_gpu": nv,
                      "traffic_bytes_per_launch": traffic_v, "fetch_counter": f_viv, "write_counter": w_viv,
                      "gather_bytes_modelled": gather, "fetch_modelled": streams / 2 + 0.998 * gather,
                      "source": f"profiles/{RND}/{VTAG}_summary.md",
                      "method": "2*(FETCH - 0.998*gather) + gather + u8 index read + WRITE"}
GTAG = os.environ.get("GOSSIP_TAG", "gossip_r01c")
g = os.path.join(OUT, f"prof_{GTAG}")
if not os.path.isdir(f"{g}_fetch"):  # keep the committed gossip entry
    json.dump(res, open(os.path.join(ROOT, "profiles", "traffic.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))
    sys.exit(0)
f_merge = last(f"{g}_fetch/run_counter_collection.csv", "FETCH_SIZE", "merge_kernel")
w_merge = last(f"{g}_write/run_counter_collection.csv", "WRITE_SIZE", "merge_kernel")
line = next(json.loads(x) for x in open(f"{g}_trace.log") if x.startswith("{") and '"metric"' in x)
n = line["config"]["members_per_gpu"]
qcap = line["config"]["queue_cap_per_queue"]
fanout = line["config"]["fanout"]
cap_t = line["config"]["record_slots_per_group"]
# coalesced streams of merge_kernel (tallied at 1/2 by FETCH_SIZE): the (sender, peer) groups'
# record slots (rumor id + decoration, 8 B per slot; one group per (sender, peer), n * fanout
# in all) with their counts (4 B per group).  The merge no longer reads the broadcast queues
# (re-queues go to the pending lists, written, not read).
stream_merge = n * fanout * (cap_t * 8 + 4)
traffic = f_merge + stream_merge / 2 + w_merge
res["gossip"] = {"kernel": "merge_kernel", "members_per_gpu": n, "traffic_bytes_per_launch": traffic,
                 "fetch_counter": f_merge, "write_counter": w_merge, "stream_bytes_modelled": stream_merge,
                 "source": f"profiles/{RND}/{GTAG}_summary.md", "method": "FETCH + stream/2 + WRITE"}
json.dump(res, open(os.path.join(ROOT, "profiles", "traffic.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
