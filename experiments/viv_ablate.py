"""Diagnostic only (not part of the product or the tests): times
vivaldi_round_kernel variants with memory streams removed, to attribute the
round time.  Results of the ablated variants are numerically meaningless."""
import ctypes as C
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from ruserf_amd import CoordinateClients, CoordinateOptions  # noqa: E402
from ruserf_amd._lib import lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64_000_000
L = lib()
L.rsf_vivaldi_round_ablate.restype = C.c_int
L.rsf_vivaldi_round_ablate.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
torch.cuda.set_stream(torch.cuda.Stream())
s = torch.cuda.current_stream()
g = CoordinateClients(n, 16, CoordinateOptions())
g.set_stream(s.cuda_stream)
g.round(0)  # fills the context's probe buffers the ablated observe kernels read
out = {}
for mask, name in [(0, "full"), (1, "no_peer_gather"), (2, "no_filter"), (4, "no_window"), (8, "no_self_row_read"),
                   (16, "no_row_write"), (32, "no_probe_inputs"), (1 | 2 | 4, "self_row_only"), (63, "compute_only"),
                   (0, "full_again")]:
    for r in range(3):
        L.rsf_vivaldi_round_ablate(g._h, r, mask)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for r in range(5):
        L.rsf_vivaldi_round_ablate(g._h, 3 + r, mask)
    e1.record(s)
    torch.cuda.synchronize()
    out[name] = e0.elapsed_time(e1) / 5
print(json.dumps(out))
