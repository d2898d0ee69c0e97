"""ctypes signatures of the gossip half of include/ruserf_amd.h."""
import ctypes as C

from ._lib import P8, P16, P32, P64, PI32, VP


class RsfGossipCfg(C.Structure):
    _fields_ = [("n_members", C.c_uint64), ("shard_lo", C.c_uint64), ("shard_hi", C.c_uint64),
                ("n_subjects", C.c_uint32), ("queue_cap", C.c_uint32), ("event_buffer_size", C.c_uint32),
                ("query_buffer_size", C.c_uint32), ("slot_k", C.c_uint32), ("fanout", C.c_uint32),
                ("gossip_limit", C.c_uint32), ("gossip_overhead", C.c_uint32), ("retransmit_mult", C.c_uint32),
                ("max_refute", C.c_uint32), ("max_rumors", C.c_uint32), ("max_user_event_size", C.c_uint32),
                ("seed", C.c_uint64), ("queue_depth", C.c_uint32 * 3), ("query_size_limit", C.c_uint32)]


def declare(L):
    i = C.c_int

    def sig(name, args):
        # a library built before a function existed (an A/B variant) lacks its symbol: calling
        # that function then fails loudly; tests/test_capi.py checks the shipped library
        # exports every declared symbol
        fn = getattr(L, name, None)
        if fn is None:
            return
        fn.restype = i
        fn.argtypes = args

    sig("rsf_gossip_create", [C.POINTER(VP), C.POINTER(RsfGossipCfg), i])
    sig("rsf_gossip_destroy", [VP])
    sig("rsf_gossip_set_stream", [VP, VP])
    sig("rsf_gossip_sync", [VP])
    sig("rsf_gossip_set_subjects", [VP, P32])
    sig("rsf_gossip_init_views", [VP, P8, P8, P64])
    sig("rsf_gossip_set_view", [VP, C.c_uint64, C.c_uint32, C.c_uint8, C.c_uint8, C.c_uint64])
    sig("rsf_gossip_set_alive", [VP, P8])
    sig("rsf_gossip_set_clocks", [VP, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64])
    sig("rsf_gossip_set_min_times", [VP, C.c_uint64, C.c_uint64, C.c_uint64])
    sig("rsf_gossip_set_serf_state", [VP, C.c_uint64, C.c_uint8])
    sig("rsf_gossip_apply_batch", [VP, VP, C.c_uint64, PI32, P64])
    sig("rsf_gossip_round", [VP, C.c_uint32, VP, C.c_uint32, VP, C.c_uint32])
    sig("rsf_gossip_round_begin", [VP, C.c_uint32, VP, C.c_uint32, VP, C.c_uint32])
    sig("rsf_gossip_rumor_block", [VP, C.POINTER(VP), P64])
    sig("rsf_gossip_round_emit", [VP, C.c_uint32, P64])
    sig("rsf_gossip_send_buffer", [VP, C.POINTER(VP), P64])
    sig("rsf_gossip_round_merge", [VP, VP, C.c_uint64])
    sig("rsf_gossip_round_merge_runs", [VP, VP, C.POINTER(C.c_uint64), C.c_uint32])
    sig("rsf_gossip_check_runs", [VP, C.POINTER(C.c_int)])
    sig("rsf_gossip_dump_members", [VP, P64, P64, P64, P64, P32, P8])
    sig("rsf_gossip_dump_view", [VP, P64, P8, P8, P32])
    sig("rsf_gossip_dump_view_rows", [VP, C.c_uint64, C.c_uint64, P64, P8, P8, P32])
    sig("rsf_gossip_reap", [VP, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32])
    sig("rsf_gossip_set_now", [VP, C.c_uint32])
    sig("rsf_gossip_dump_queues", [VP, P32, P32, P16, P16, P32])
    sig("rsf_gossip_deep_stats", [VP, P64, P64])
    sig("rsf_gossip_dump_queues_width", [VP, C.c_uint32, P32, P32, P16, P16, P32, P32])
    sig("rsf_gossip_dump_buffers", [VP, P64, P32, P64, P64, P32, P32])
    sig("rsf_gossip_dump_rumors", [VP, C.c_uint32, C.c_uint32, VP])
    sig("rsf_gossip_dump_refutes", [VP, P32, P64])
    sig("rsf_gossip_last_round_stats", [VP, P64, P64])
    sig("rsf_gossip_set_profiling", [VP, i])
    sig("rsf_gossip_phase_times", [VP, C.POINTER(C.c_double), P32])
    sig("rsf_gossip_totals", [VP, P64])
    sig("rsf_gossip_push_pull", [VP, VP, C.c_uint64, C.c_uint32])
    sig("rsf_gossip_push_pull_device", [VP, VP, C.c_uint64, C.c_uint32])
    sig("rsf_gossip_action_status", [VP, PI32, C.c_uint32])
    sig("rsf_gossip_deep_class_stats", [VP, P64])
    sig("rsf_gossip_deep_full_items", [VP, P64, P64])
    sig("rsf_gossip_dump_tails", [VP, C.c_uint32, P32, P32])
    sig("rsf_gossip_queue_lengths", [VP, P32])
    sig("rsf_gossip_dump_queues_rows", [VP, C.c_uint64, C.c_uint64, C.c_uint32, P32, P32, P16, P16, P32])
    sig("rsf_gossip_checker_occupancy", [VP, P32, P32, P32, P32])
    sig("rsf_gossip_check_queues", [VP, C.c_uint32, C.c_uint32, C.c_uint32, P64, P64, P64])
    sig("rsf_gossip_check_queues_phase", [VP, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32])
    sig("rsf_gossip_checker_stats", [VP, P64, P64, P64, i])
    sig("rsf_gossip_set_checker", [VP, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32])
    sig("rsf_gossip_dump_pruned", [VP, P32, P32])
    sig("rsf_gossip_flush", [VP])
    sig("rsf_gossip_pruned_total", [VP, C.c_int, C.POINTER(C.c_uint64)])
    sig("rsf_gossip_set_delivery_log", [VP, C.c_uint32])
    sig("rsf_gossip_bucket_buffers", [VP, C.c_uint32, C.POINTER(VP), C.POINTER(VP), P64])
    sig("rsf_gossip_round_emit_buckets", [VP, C.c_uint32])
    sig("rsf_gossip_round_merge_buckets", [VP, C.c_uint32])
    sig("rsf_gossip_bucket_status", [VP, C.POINTER(C.c_int)])
    sig("rsf_gossip_dump_deliveries", [VP, VP, C.c_uint64, P64])
    sig("rsf_gossip_enable_snapshot", [VP, i])
    sig("rsf_gossip_snapshot_encode", [VP, C.c_uint64, C.c_uint64, VP, VP, C.c_uint64, P64])
    sig("rsf_gossip_restart", [VP, P32, C.c_uint32, P8, P64, C.POINTER(C.c_int32)])
    sig("rsf_gossip_dump_snapshot", [VP, P32, P64])
    sig("rsf_gossip_reconnect", [VP, C.c_uint32, VP])
    sig("rsf_gossip_debug_canaries", [VP, C.POINTER(C.c_int)])
