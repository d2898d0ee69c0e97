"""ctypes bindings for the CPU oracle (oracle/liboracle.so).

Test infrastructure only: used by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the CHECKER.  The product package ruserf_amd
never imports this module.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")

MAX_DIM = 16
MAX_WINDOW = 64
MAX_FILTER = 8


class CoordOpts(C.Structure):
    _fields_ = [("dimensionality", C.c_uint32), ("adjustment_window_size", C.c_uint32),
                ("latency_filter_size", C.c_uint32), ("_pad", C.c_uint32),
                ("vivaldi_error_max", C.c_double), ("vivaldi_ce", C.c_double),
                ("vivaldi_cc", C.c_double), ("height_min", C.c_double),
                ("gravity_rho", C.c_double)]


class Coord(C.Structure):
    _fields_ = [("portion", C.c_double * MAX_DIM), ("dim", C.c_uint32), ("_pad", C.c_uint32),
                ("error", C.c_double), ("adjustment", C.c_double), ("height", C.c_double)]


class Rng(C.Structure):
    _fields_ = [("key", C.c_uint32 * 2), ("member", C.c_uint32), ("round", C.c_uint32),
                ("call", C.c_uint32), ("draw", C.c_uint32)]


class Filter(C.Structure):
    _fields_ = [("s", C.c_double * (MAX_FILTER + 1)), ("len", C.c_uint32)]


class Client(C.Structure):
    _fields_ = [("coord", Coord), ("origin", Coord), ("opts", CoordOpts),
                ("adjustment_index", C.c_uint32), ("n_slots", C.c_uint32),
                ("adjustment_samples", C.c_double * MAX_WINDOW),
                ("filters", C.POINTER(Filter)), ("resets", C.c_uint64)]


class VivaldiPop(C.Structure):
    _fields_ = [("n", C.c_uint32), ("peers", C.c_uint32), ("row_stride", C.c_uint32),
                ("opts", CoordOpts), ("seed", C.c_uint64),
                ("rows_cur", C.POINTER(C.c_double)), ("rows_nxt", C.POINTER(C.c_double)),
                ("adj", C.POINTER(C.c_double)), ("adj_idx", C.POINTER(C.c_uint32)),
                ("filt", C.POINTER(C.c_double)), ("filt_len", C.POINTER(C.c_uint32)),
                ("nbr", C.POINTER(C.c_uint32)), ("resets", C.c_uint64)]


class Rumor(C.Structure):
    _fields_ = [("type", C.c_uint8), ("flags", C.c_uint8), ("msg_len", C.c_uint16),
                ("subject", C.c_uint32), ("ltime", C.c_uint64), ("key", C.c_uint64)]


P64 = C.POINTER(C.c_uint64)
P32 = C.POINTER(C.c_uint32)
PI32 = C.POINTER(C.c_int32)
P16 = C.POINTER(C.c_uint16)
P8 = C.POINTER(C.c_uint8)


class World(C.Structure):
    _fields_ = [("n", C.c_uint32), ("s", C.c_uint32), ("qcap", C.c_uint32), ("ebuf", C.c_uint32),
                ("qbuf", C.c_uint32), ("slot_k", C.c_uint32), ("fanout", C.c_uint32),
                ("limit", C.c_uint32), ("overhead", C.c_uint32), ("tx_limit", C.c_uint32),
                ("max_refute", C.c_uint32), ("seed", C.c_uint64),
                ("clock", P64), ("eclock", P64), ("qclock", P64), ("emin", P64), ("qmin", P64),
                ("digest", P64), ("alive", P8), ("serf_state", P8), ("err", P32),
                ("subj_member", P32), ("member_subj", PI32), ("refute_cnt", P32),
                ("refute_ltime", P64), ("v_ltime", P64), ("v_status", P8), ("v_kind", P8),
                ("q_rumor", P32), ("q_seq", P32), ("q_tx", P16), ("q_len", P16),
                ("q_next_seq", P32), ("eb_ltime", P64), ("eb_cnt", P32), ("eb_keys", P64),
                ("qb_ltime", P64), ("qb_cnt", P32), ("qb_ids", P32),
                ("rumors", C.POINTER(Rumor)), ("n_rumors", C.c_uint32), ("cap_rumors", C.c_uint32),
                ("merges", C.c_uint64), ("sends", C.c_uint64), ("deliveries", C.c_uint64),
                ("v_time", P32), ("now", C.c_uint32), ("q_pruned", P32), ("q_expired", P32),
                ("gen", C.c_uint32), ("rbits", C.c_uint32), ("dlog", P64), ("dcnt", P32), ("dcap", C.c_uint32),
                ("snap_bits", P32), ("snap_w", C.c_uint32), ("snap_rejoin", C.c_int32), ("snap_sn", P64),
                ("qd", C.c_uint32 * 3), ("q_hwm", P32), ("max_ue", C.c_uint32), ("query_limit", C.c_uint32),
                ("act_status", PI32), ("act_cap", C.c_uint32), ("last_n_acts", C.c_uint32),
                ("chk_period", C.c_uint32), ("chk_max", C.c_uint32), ("chk_min", C.c_uint32),
                ("chk_warn", C.c_uint32), ("chk_stats", C.c_uint64 * 9), ("q_hole", P32)]


class WorldCfg(C.Structure):
    _fields_ = [("n", C.c_uint32), ("s", C.c_uint32), ("qcap", C.c_uint32), ("ebuf", C.c_uint32),
                ("qbuf", C.c_uint32), ("slot_k", C.c_uint32), ("fanout", C.c_uint32),
                ("limit", C.c_uint32), ("overhead", C.c_uint32), ("retransmit_mult", C.c_uint32),
                ("max_refute", C.c_uint32), ("cap_rumors", C.c_uint32), ("seed", C.c_uint64),
                ("qdepth", C.c_uint32 * 3), ("max_user_event_size", C.c_uint32),
                ("query_size_limit", C.c_uint32), ("_pad", C.c_uint32)]


class Action(C.Structure):
    _fields_ = [("member", C.c_uint32), ("act", C.c_uint32), ("subject", C.c_uint32),
                ("name_len", C.c_uint32), ("payload_len", C.c_uint32), ("flags", C.c_uint32),
                ("key", C.c_uint64)]


class MlEvent(C.Structure):
    _fields_ = [("subject", C.c_uint32), ("kind", C.c_uint32), ("set_alive", C.c_uint32),
                ("_pad", C.c_uint32)]


UEvent = None


class _UEvent(C.Structure):
    _fields_ = [("name", C.c_uint32), ("ltime", C.c_uint64), ("payload", C.c_uint64)]


UEvent = _UEvent


class MEvent(C.Structure):
    _fields_ = [("group", C.c_uint32), ("node", C.c_uint32), ("type", C.c_uint32), ("member", C.c_uint32)]


LOG_CC = 1  # delivery-log flags word (oracle.h ORC_LOG_CC / ORC_LOG_MEMBER)
LOG_MEMBER = 0x100

# enums (oracle.h)
OK, ERR_DIM, ERR_COORD, ERR_RTT = 0, 1, 2, 3
ST_NONE, ST_ALIVE, ST_LEAVING, ST_LEFT, ST_FAILED = 0, 1, 2, 3, 4
K_UNKNOWN, K_JOIN, K_LEAVE, K_KNOWN = 0, 1, 2, 3
F_REBROADCAST, F_REFUTE, F_PRUNE, F_DELIVER, F_MEMBER_EVENT = 1, 2, 4, 8, 16
ACT_JOIN_SELF, ACT_LEAVE_SELF, ACT_FORCE_LEAVE, ACT_USER_EVENT, ACT_QUERY = 1, 2, 3, 4, 5
ML_JOIN, ML_LEAVE, ML_UPDATE = 1, 2, 3

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    L = C.CDLL(LIB_PATH)
    L.orc_philox4x32.argtypes = [P32, P32, P32]
    L.orc_coord_opts_default.argtypes = [C.POINTER(CoordOpts)]
    L.orc_coord_with_options.argtypes = [C.POINTER(CoordOpts), C.POINTER(Coord)]
    L.orc_coord_is_valid.argtypes = [C.POINTER(Coord)]
    L.orc_coord_distance_ns.argtypes = [C.POINTER(Coord), C.POINTER(Coord)]
    L.orc_coord_distance_ns.restype = C.c_uint64
    L.orc_coord_raw_distance.argtypes = [C.POINTER(Coord), C.POINTER(Coord)]
    L.orc_coord_raw_distance.restype = C.c_double
    L.orc_magnitude.argtypes = [C.POINTER(C.c_double), C.c_uint32]
    L.orc_magnitude.restype = C.c_double
    L.orc_unit_vector_at.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_uint32,
                                     C.POINTER(C.c_double), C.POINTER(Rng)]
    L.orc_unit_vector_at.restype = C.c_double
    L.orc_apply_force_in_place.argtypes = [C.POINTER(Coord), C.c_double, C.c_double,
                                           C.POINTER(Coord), C.POINTER(Rng)]
    L.orc_as_secs_f64.argtypes = [C.c_uint64]
    L.orc_as_secs_f64.restype = C.c_double
    L.orc_client_init.argtypes = [C.POINTER(Client), C.POINTER(CoordOpts), C.c_uint32]
    L.orc_client_free.argtypes = [C.POINTER(Client)]
    L.orc_client_set_coordinate.argtypes = [C.POINTER(Client), C.POINTER(Coord)]
    L.orc_client_forget_node.argtypes = [C.POINTER(Client), C.c_uint32]
    L.orc_client_latency_filter.argtypes = [C.POINTER(Client), C.c_uint32, C.c_double]
    L.orc_client_latency_filter.restype = C.c_double
    L.orc_client_update.argtypes = [C.POINTER(Client), C.c_uint32, C.POINTER(Coord), C.c_uint64,
                                    C.POINTER(Rng), C.POINTER(Coord)]
    L.orc_row_stride.argtypes = [C.c_uint32]
    L.orc_row_stride.restype = C.c_uint32
    L.orc_vivaldi_pop_init.argtypes = [C.POINTER(VivaldiPop), C.c_uint32, C.c_uint32,
                                       C.POINTER(CoordOpts), C.c_uint64]
    L.orc_vivaldi_pop_free.argtypes = [C.POINTER(VivaldiPop)]
    L.orc_vivaldi_pop_rounds.argtypes = [C.POINTER(VivaldiPop), C.c_uint32, C.c_uint32, C.c_int]
    L.orc_vivaldi_pop_median_rel_error.argtypes = [C.POINTER(VivaldiPop)]
    L.orc_vivaldi_pop_rounds_stale.argtypes = [C.POINTER(VivaldiPop), C.c_uint32, C.c_uint32, C.c_int,
                                               C.POINTER(C.c_double), C.c_uint32, C.c_uint32]
    L.orc_vivaldi_pop_median_rel_error.restype = C.c_double
    L.orc_vivaldi_probe.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, P32, C.c_uint32, C.c_uint32,
                                    P32, P64]
    L.orc_true_position.argtypes = [C.c_uint64, C.c_uint32, C.POINTER(C.c_double),
                                    C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.orc_gen_neighbors.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, P32]
    L.orc_world_init.argtypes = [C.POINTER(World), C.POINTER(WorldCfg)]
    L.orc_world_free.argtypes = [C.POINTER(World)]
    L.orc_retransmit_limit.argtypes = [C.c_uint32, C.c_uint64]
    L.orc_retransmit_limit.restype = C.c_uint32
    L.orc_handle_join_intent.argtypes = [C.POINTER(World), C.c_uint32, C.c_uint32, C.c_uint64]
    L.orc_handle_leave_intent.argtypes = [C.POINTER(World), C.c_uint32, C.c_uint32, C.c_uint64,
                                          C.c_int, P64]
    L.orc_handle_node_join.argtypes = [C.POINTER(World), C.c_uint32, C.c_uint32]
    L.orc_handle_node_leave.argtypes = [C.POINTER(World), C.c_uint32, C.c_uint32]
    L.orc_handle_node_update.argtypes = [C.POINTER(World), C.c_uint32, C.c_uint32]
    L.orc_handle_user_event.argtypes = [C.POINTER(World), C.c_uint32, C.c_uint64, C.c_uint64]
    L.orc_handle_query.argtypes = [C.POINTER(World), C.c_uint32, C.c_uint64, C.c_uint32, C.c_int]
    L.orc_upsert_intent.argtypes = [C.POINTER(World), C.c_uint32, C.c_uint32, C.c_uint8, C.c_uint64]
    L.orc_queue_insert.argtypes = [C.POINTER(World), C.c_uint32, C.c_uint32, C.c_uint32]
    L.orc_queue_get_broadcasts.argtypes = [C.POINTER(World), C.c_uint32, C.c_uint32, C.c_uint32,
                                           P32, C.c_uint32, P32]
    L.orc_queue_get_broadcasts.restype = C.c_uint32
    L.orc_msg_len.argtypes = [C.c_uint8, C.c_uint64, C.c_uint32, C.c_uint32]
    L.orc_msg_len.restype = C.c_uint32
    L.orc_digest_mix.argtypes = [C.c_uint64, C.c_uint64]
    L.orc_digest_mix.restype = C.c_uint64
    L.orc_world_round.argtypes = [C.POINTER(World), C.c_uint32, C.POINTER(MlEvent), C.c_uint32,
                                  C.POINTER(Action), C.c_uint32]
    L.orc_world_round_mt.argtypes = [C.POINTER(World), C.c_uint32, C.POINTER(MlEvent), C.c_uint32,
                                     C.POINTER(Action), C.c_uint32, C.c_int]
    L.orc_world_set_delivery_log.argtypes = [C.POINTER(World), C.c_uint32]
    L.orc_handle_user_event_cc.argtypes = [C.POINTER(World), C.c_uint32, C.c_uint64, C.c_uint64, C.c_int]
    L.orc_rumor_index.argtypes = [C.POINTER(World), C.c_uint32]
    L.orc_rumor_index.restype = C.c_uint32
    L.orc_rumor_live.argtypes = [C.POINTER(World), C.c_uint32]
    L.orc_rumor_live.restype = C.c_int
    L.orc_pick_peers.argtypes = [C.c_uint64, C.c_uint32, P8, C.c_uint32, C.c_uint32, C.c_uint32, P32]
    L.orc_pick_peers.restype = C.c_uint32
    L.orc_merge_remote_state.argtypes = [C.POINTER(World), C.c_uint32, C.POINTER(PPState), C.c_int, C.c_int]
    L.orc_push_pull.argtypes = [C.POINTER(World), P32, P32, C.c_uint32, C.c_int, C.c_int]
    L.orc_states_len.argtypes = [C.POINTER(World), C.c_uint32]
    L.orc_states_len.restype = C.c_uint64
    L.orc_world_action_status.argtypes = [C.POINTER(World), PI32, C.c_uint32]
    L.orc_user_event_check.argtypes = [C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32]
    L.orc_user_event_check.restype = C.c_int32
    L.orc_query_check.argtypes = [C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32]
    L.orc_query_check.restype = C.c_int32
    L.orc_check_queues.argtypes = [C.POINTER(World), C.c_uint32, C.c_uint32, C.c_uint32, P64]
    L.orc_check_queues.restype = None
    L.orc_check_queues_phase.argtypes = [C.POINTER(World), C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                         C.c_uint32, P64]
    L.orc_check_queues_phase.restype = None
    L.orc_world_set_checker.argtypes = [C.POINTER(World), C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
    L.orc_world_set_checker.restype = None
    L.orc_reap.argtypes = [C.POINTER(World), C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
    L.orc_varint_len.argtypes = [C.c_uint64]
    L.orc_varint_len.restype = C.c_uint32
    L.orc_varint_encode.argtypes = [C.c_uint64, P8]
    L.orc_varint_encode.restype = C.c_uint32
    L.orc_varint_decode.argtypes = [P8, C.c_uint64, P64, C.POINTER(C.c_int)]
    L.orc_varint_decode.restype = C.c_uint32
    L.orc_coord_encode.argtypes = [C.POINTER(C.c_double), C.c_uint32, P8]
    L.orc_coord_encode.restype = C.c_uint32
    L.orc_coord_decode.argtypes = [P8, C.c_uint64, C.c_uint32, C.POINTER(C.c_double), P32]
    L.orc_coord_decode.restype = C.c_int
    L.orc_wire_frame_len.argtypes = [C.c_void_p]
    L.orc_wire_frame_len.restype = C.c_uint32
    L.orc_wire_encode.argtypes = [C.c_void_p, P8, P8]
    L.orc_wire_encode.restype = C.c_uint32
    L.orc_wire_decode.argtypes = [P8, C.c_uint64, C.c_uint64, C.c_void_p]
    L.orc_coalesce_user_events.argtypes = [C.POINTER(UEvent), C.c_uint32, C.POINTER(UEvent)]
    L.orc_coalesce_user_events.restype = C.c_uint32
    L.orc_member_coalesce.argtypes = [C.POINTER(C.c_uint8), C.c_uint32, C.POINTER(MEvent), C.c_uint64,
                                      C.POINTER(MEvent)]
    L.orc_member_coalesce.restype = C.c_uint64
    L.orc_swim_init.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, P32, P32, P8, P32,
                                C.c_uint32]
    L.orc_swim_free.argtypes = [C.c_void_p]
    L.orc_swim_free.restype = None
    L.orc_swim_set_left.argtypes = [C.c_void_p, C.c_uint64, C.c_uint8]
    L.orc_swim_set_left.restype = None
    L.orc_swim_apply.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.POINTER(C.c_int32), P32]
    L.orc_swim_apply.restype = None
    L.orc_swim_tick.argtypes = [C.c_void_p, C.c_uint32]
    L.orc_swim_tick.restype = C.c_uint64
    L.orc_swim_dump.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, P8, P32, P32, P8, P32]
    L.orc_swim_dump.restype = None
    L.orc_snapshot_replay.argtypes = [P8, C.c_uint64, C.c_int, C.c_uint32, P32, P64]
    L.orc_snapshotter_open.argtypes = [C.POINTER(Snapshotter), C.c_uint32, P8, C.c_uint64, C.c_uint64, C.c_int]
    L.orc_snapshotter_free.argtypes = [C.POINTER(Snapshotter)]
    L.orc_snapshotter_free.restype = None
    for f in ("orc_snapshotter_user_event", "orc_snapshotter_query", "orc_snapshotter_update_clock"):
        getattr(L, f).argtypes = [C.POINTER(Snapshotter), C.c_uint64]
        getattr(L, f).restype = None
    L.orc_snapshotter_member_event.argtypes = [C.POINTER(Snapshotter), C.c_uint32, C.c_uint32, C.c_uint64]
    L.orc_snapshotter_member_event.restype = None
    L.orc_snapshotter_leave.argtypes = [C.POINTER(Snapshotter)]
    L.orc_snapshotter_leave.restype = None
    L.orc_world_enable_snapshot.argtypes = [C.POINTER(World), C.c_int]
    L.orc_world_snapshot_encode.argtypes = [C.POINTER(World), C.c_uint32, P8]
    L.orc_world_snapshot_encode.restype = C.c_uint64
    L.orc_world_restart.argtypes = [C.POINTER(World), C.c_uint32, P8, C.c_uint64]
    L.orc_world_reconnect.argtypes = [C.POINTER(World), C.c_uint32, P32]
    L.orc_world_reconnect.restype = C.c_uint32
    L.orc_reconnect_prob.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
    L.orc_reconnect_prob.restype = C.c_float
    _lib = L
    return L


class Snapshotter(C.Structure):
    _fields_ = [("buf", P8), ("len", C.c_uint64), ("cap", C.c_uint64), ("offset", C.c_uint64),
                ("min_compact", C.c_uint64), ("compactions", C.c_uint64), ("alive", P32), ("s", C.c_uint32),
                ("last_clock", C.c_uint64), ("last_event_clock", C.c_uint64), ("last_query_clock", C.c_uint64),
                ("leaving", C.c_int), ("rejoin", C.c_int)]


class OrcSwim(C.Structure):
    _fields_ = [("lo", C.c_uint64), ("n_loc", C.c_uint64), ("S", C.c_uint32), ("k", C.c_uint32),
                ("timeout", C.c_uint32 * 5), ("_pad", C.c_uint32)] + \
               [(f, C.c_void_p) for f in ("state", "inc", "change", "nconf", "accuser", "self_inc", "left",
                                          "subject_member")]


class OracleSwim:
    """The oracle's memberlist SWIM model (orc_swim_*), same surface as ruserf_amd.swim.SwimState."""

    def __init__(self, lo, n_loc, S, k, timeouts, subject_member, state0, inc0, self_inc0=1):
        self.L, self.S, self.lo, self.n_loc = lib(), S, lo, n_loc
        self.w = OrcSwim()
        t = np.ascontiguousarray(timeouts, np.uint32)
        sm = np.ascontiguousarray(subject_member, np.uint32)
        st = np.ascontiguousarray(state0, np.uint8)
        ic = np.ascontiguousarray(inc0, np.uint32)
        rc = self.L.orc_swim_init(C.byref(self.w), lo, n_loc, S, k, t.ctypes.data_as(P32), sm.ctypes.data_as(P32),
                                  st.ctypes.data_as(P8), ic.ctypes.data_as(P32), self_inc0)
        assert rc == 0

    def close(self):
        self.L.orc_swim_free(C.byref(self.w))

    def set_left(self, member, left=True):
        self.L.orc_swim_set_left(C.byref(self.w), member, 1 if left else 0)

    def apply(self, msgs, now):
        n = len(msgs)
        f = np.zeros(n, np.int32)
        r = np.zeros(n, np.uint32)
        m = np.ascontiguousarray(msgs)
        self.L.orc_swim_apply(C.byref(self.w), m.ctypes.data, n, now, f.ctypes.data_as(C.POINTER(C.c_int32)),
                              r.ctypes.data_as(P32))
        return f, r

    def tick(self, now):
        return int(self.L.orc_swim_tick(C.byref(self.w), now))

    def dump(self, first=0, count=None):
        count = self.n_loc - first if count is None else count
        S = self.S
        st, inc, ch = np.zeros(count * S, np.uint8), np.zeros(count * S, np.uint32), np.zeros(count * S, np.uint32)
        nc, si = np.zeros(count * S, np.uint8), np.zeros(count, np.uint32)
        self.L.orc_swim_dump(C.byref(self.w), first, count, st.ctypes.data_as(P8), inc.ctypes.data_as(P32),
                             ch.ctypes.data_as(P32), nc.ctypes.data_as(P8), si.ctypes.data_as(P32))
        return {"state": st.reshape(count, S), "incarnation": inc.reshape(count, S),
                "change": ch.reshape(count, S), "n_confirm": nc.reshape(count, S), "self_incarnation": si}


class PPState(C.Structure):
    """orc_pp_state: a member's local_state as merge_remote_state reads it"""
    _fields_ = [("clock", C.c_uint64), ("eclock", C.c_uint64), ("qclock", C.c_uint64),
                ("v_ltime", C.POINTER(C.c_uint64)), ("v_status", C.POINTER(C.c_uint8)),
                ("v_kind", C.POINTER(C.c_uint8)), ("eb_ltime", C.POINTER(C.c_uint64)),
                ("eb_cnt", C.POINTER(C.c_uint32)), ("eb_keys", C.POINTER(C.c_uint64))]


def default_opts(**kw):
    o = CoordOpts()
    lib().orc_coord_opts_default(C.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def coord(opts, portion=None, error=None, adjustment=None, height=None):
    c = Coord()
    lib().orc_coord_with_options(C.byref(opts), C.byref(c))
    if portion is not None:
        c.dim = len(portion)
        for i, v in enumerate(portion):
            c.portion[i] = v
    if error is not None:
        c.error = error
    if adjustment is not None:
        c.adjustment = adjustment
    if height is not None:
        c.height = height
    return c


def rng(seed=0x5EED5EED, member=0, round_=0):
    r = Rng()
    r.key[0] = seed & 0xFFFFFFFF
    r.key[1] = (seed >> 32) & 0xFFFFFFFF
    r.member = member
    r.round = round_
    return r


def arr(ptr, n, dtype):
    """numpy view of an oracle-owned C array"""
    if n == 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).view(dtype)


def ptr(a, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def member_coalesce(last, events):
    """oracle MemberEventCoalescer flush over (group, node, type, member) rows; last: the
    [n_groups][n_nodes] u8 table, updated in place -> flushed rows (numpy structured)"""
    from ruserf_amd.coalesce import MEMBER_EVENT_DTYPE
    ev = np.ascontiguousarray(events, dtype=MEMBER_EVENT_DTYPE)
    n = len(ev)
    out = np.zeros(max(1, n), MEMBER_EVENT_DTYPE)
    assert last.flags.c_contiguous and last.dtype == np.uint8
    k = lib().orc_member_coalesce(last.ctypes.data_as(C.POINTER(C.c_uint8)), last.shape[1],
                                  ev.ctypes.data_as(C.POINTER(MEvent)), n, out.ctypes.data_as(C.POINTER(MEvent)))
    return out[:k].copy()
