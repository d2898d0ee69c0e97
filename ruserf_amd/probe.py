"""memberlist's probe loop feeding the coordinate clients and the failure detector
(SURVEY §8(f)3).  memberlist is not vendored by the reference: parity unpinned.

Per round r, on one stream, with every input and output resident in HBM:
  1. probe      -- member m probes neighbour slot r mod P of its fixed probe list
                   (memberlist's round-robin probe, the latency-filter slots of
                   CoordinateClient); acked when both processes are up
  2. ack        -- wire=True: the target's SerfDelegate::ack_payload bytes
                   ([PING_VERSION][Coordinate], delegate.rs:659-701) are built for every
                   acked probe and fed to notify_ping_complete (delegate.rs:704-779,
                   rsf_vivaldi_observe_acks); wire=False: the coordinate rows are read from
                   the table directly (rsf_vivaldi_observe), the same update
  3. suspicion  -- a probe without ack runs suspectNode{target} at the prober
                   (rsf_swim_probe_failures) when a SwimState is attached
"""
import torch

from .coordinate import CoordinateClients
from .swim import SwimState


class ProbeLoop:
    def __init__(self, clients: CoordinateClients, swim: SwimState = None, wire=True, stream=None):
        self.v, self.swim, self.wire = clients, swim, wire
        self.dev = torch.device("cuda", torch.cuda.current_device())
        # a stream of its own: torch's default stream has the NULL handle, which the C ABI
        # reads as "each context's own stream", and then the probe (coordinate context) and
        # the suspicion (SWIM context) would not be ordered
        self.stream = stream if stream is not None and stream.cuda_stream else torch.cuda.Stream()
        clients.set_stream(self.stream.cuda_stream)
        if swim is not None:
            swim.set_stream(self.stream.cuda_stream)
        n = clients.hi - clients.lo
        self.n = n
        self.peer = torch.empty(n, dtype=torch.int32, device=self.dev)
        self.rtt = torch.empty(n, dtype=torch.int64, device=self.dev)
        self.acked = torch.empty(n, dtype=torch.uint8, device=self.dev)
        self.status = torch.empty(n, dtype=torch.int32, device=self.dev)
        self.flags = torch.zeros(n, dtype=torch.int32, device=self.dev)
        if wire:
            plen = 1 + 28 + 8 * clients.dim  # PING_VERSION + Coordinate encoding
            self.members = torch.arange(clients.lo, clients.hi, dtype=torch.int32, device=self.dev)
            self.slots = torch.empty(n, dtype=torch.int32, device=self.dev)
            self.off = torch.empty(n + 1, dtype=torch.int64, device=self.dev)
            self.payload = torch.empty(n * plen, dtype=torch.uint8, device=self.dev)

    def round(self, r, up, now=None):
        """One probe round; `up` = uint8 CUDA tensor of every member's process liveness."""
        v = self.v
        self.stream.wait_stream(torch.cuda.current_stream())  # `up` and the caller's prior work
        with torch.cuda.stream(self.stream):
            v.probe(r, up.data_ptr(), self.peer.data_ptr(), self.rtt.data_ptr(), self.acked.data_ptr())
            slot = r % v.peer_slots
            if self.wire:
                self.slots.fill_(slot)
                v.probe_acks(self.peer.data_ptr(), self.acked.data_ptr(), self.off.data_ptr(),
                             self.payload.data_ptr(), self.payload.numel())
                v.observe_acks_device(self.members.data_ptr(), self.slots.data_ptr(), self.payload.data_ptr(),
                                      self.off.data_ptr(), self.rtt.data_ptr(), self.n, self.status.data_ptr(), r)
            else:
                v.observe(slot, self.peer.data_ptr(), self.rtt.data_ptr(), self.status.data_ptr(), r)
            if self.swim is not None:
                self.swim.probe_failures(self.peer.data_ptr(), self.acked.data_ptr(), up.data_ptr(),
                                         r if now is None else now, self.flags.data_ptr())
