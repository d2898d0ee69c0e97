"""The MergeDelegate hook (core/src/delegate/merge.rs:13-28) on the engine's host side.

memberlist asks the merge delegate twice (core/src/serf/delegate.rs:580-630):
  * `notify_alive` -> `notify_merge([member])` before an alive node is applied;
  * `notify_merge(peers)` before a join's promised push/pull merges the remote nodes.
An `Err` cancels that merge.  In the engine, memberlist's decisions arrive as host
lists -- the round's `rsf_ml_event` JOIN rows and the `is_join` push/pull pairs -- so
the hook runs here, before those lists are handed to the kernels: a cancelled alive
node produces no NotifyJoin (no `handle_node_join`), a cancelled join merge produces
no push/pull pair.  It is not consulted for anti-entropy push/pull, as in the reference.
"""
from dataclasses import dataclass
from typing import Callable, Iterable, Sequence

import numpy as np

from .gossip import ML_JOIN, PP_PAIR_DTYPE


class MergeCanceled(Exception):
    """Raised by a delegate to cancel a merge (the reference's `Err(..)`)."""


@dataclass(frozen=True)
class Member:
    """types::Member as the hook sees it: the subject slot, its member id, its status
    (MemberStatus numbering, RSF_STATUS_*)."""
    subject: int
    member: int
    status: int = 1


class MergeDelegate:
    """Override notify_merge; raise MergeCanceled (or any exception) to cancel."""

    def notify_merge(self, members: Sequence[Member]) -> None:
        return None


class DefaultMergeDelegate(MergeDelegate):
    """DefaultMergeDelegate (merge.rs:31-57): accepts every merge."""


def _accepts(delegate: MergeDelegate, members: Sequence[Member]) -> bool:
    try:
        delegate.notify_merge(list(members))
    except Exception:  # the reference maps any delegate error to a cancelled merge
        return False
    return True


def filter_alive_events(delegate: MergeDelegate, ml: np.ndarray, subject_member: np.ndarray) -> np.ndarray:
    """The round's memberlist events with the JOINs whose notify_alive -> notify_merge
    was cancelled removed (other events pass unchanged, order kept)."""
    if delegate is None or len(ml) == 0:
        return ml
    keep = np.ones(len(ml), dtype=bool)
    for i, e in enumerate(ml):
        if int(e["kind"]) != ML_JOIN:
            continue
        s = int(e["subject"])
        keep[i] = _accepts(delegate, [Member(s, int(subject_member[s]))])
    return ml[keep]


def filter_join_push_pull(delegate: MergeDelegate, pairs: np.ndarray,
                          remote_members: Callable[[int], Iterable[Member]]) -> np.ndarray:
    """Join push/pull pairs (PP_PAIR_DTYPE) whose notify_merge over the sender's nodes
    (remote_members(sender)) was accepted."""
    pairs = np.ascontiguousarray(pairs, dtype=PP_PAIR_DTYPE)
    if delegate is None or len(pairs) == 0:
        return pairs
    keep = np.array([_accepts(delegate, list(remote_members(int(p["sender"])))) for p in pairs], dtype=bool)
    return pairs[keep]
