"""ruserf_amd — MI355X-native engine for ruserf's data-parallel gossip round.

Host-side mirror of the reference's operator surface for the hot path
(Vivaldi CoordinateClient, the Lamport-clock member-state merge and the
retransmit-limited event/query dissemination) over hand-written HIP kernels
for gfx950 exposed through the C ABI in include/ruserf_amd.h.
"""
from ._lib import EngineError, declared_symbols, lib  # noqa: F401
from .coordinate import (Coordinate, CoordinateClients, CoordinateError,  # noqa: F401
                         CoordinateOptions)

__version__ = "0.1.0"
from . import gossip, swim, workload  # noqa: F401,E402
from .gossip import GossipConfig, GossipEngine  # noqa: F401,E402
