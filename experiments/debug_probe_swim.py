import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np, torch
import oracle_ffi as O
from ruserf_amd import CoordinateClients, CoordinateOptions
from ruserf_amd import swim as SW
from ruserf_amd.probe import ProbeLoop
n, peers, rounds, k = 2000, 16, 4, 2
rng = np.random.default_rng(3)
up_np = np.ones(n, np.uint8); up_np[rng.choice(n, int(n * 0.2), replace=False)] = 0
up = torch.from_numpy(up_np).cuda()
subj = np.arange(n, dtype=np.uint32); st0 = np.zeros(n, np.uint8); inc0 = np.ones(n, np.uint32)
cfg = SW.SwimConfig(n_members=n, n_subjects=n, suspicion_k=k, suspicion_min=3, suspicion_max=9)
sw = SW.SwimState(cfg); sw.set_subjects(subj); sw.init(st0, inc0, self_incarnation=1)
o = O.OracleSwim(0, n, n, k, sw.timeouts, subj, st0, inc0, 1)
g = CoordinateClients(n, peers, CoordinateOptions(), seed=0x5EED5EED)
loop = ProbeLoop(g, swim=sw, wire=True)
for r in range(rounds):
    before = o.dump(); gb = sw.dump()
    loop.round(r, up, now=r); torch.cuda.synchronize()
    peer = loop.peer.cpu().numpy(); acked = loop.acked.cpu().numpy().astype(bool)
    msgs = [(m, peer[m], before["incarnation"][m, peer[m]], m, SW.MSG_SUSPECT, 0) for m in range(n)
            if not acked[m] and up_np[m] and peer[m] != m]
    msgs = np.array(msgs, dtype=SW.MSG_DTYPE)
    fo, _ = o.apply(msgs, r)
    fg = loop.flags.cpu().numpy()
    want = np.zeros(n, np.int32); want[msgs["receiver"]] = fo
    bad = np.nonzero(fg != want)[0]
    print("round", r, "msgs", len(msgs), "bad", len(bad))
    for m in bad[:8]:
        t = peer[m]
        print(" m", m, "t", t, "up_m", up_np[m], "up_t", up_np[t], "acked", acked[m], "gpu", fg[m], "want", want[m],
              "state before o/g", before["state"][m, t], gb["state"][m, t], "nconf", before["n_confirm"][m, t])
    sw.tick(r); o.tick(r)
