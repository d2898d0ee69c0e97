"""Writes tests/golden/reference_kats.json: the known-answer vectors held by
al8n/ruserf's own unit tests for the hot path, transcribed as data (inputs and
expected outputs) with the file:line each one comes from.

The reference is Rust and cannot be compiled or run in this container (no
cargo/rustc, no vendored crates), so these transcribed test vectors are what
pins the CPU oracle (oracle/oracle.c).  Run:  python tests/golden/make_golden.py
"""
import json
import os
import struct

HERE = os.path.dirname(os.path.abspath(__file__))


def i64_wrapping_mul_as_u64(p_f64):
    # Duration::from_nanos((p as i64).wrapping_mul(1e9 as i64) as u64)
    # coordinate.rs:931; `f64 as i64` saturates.
    if p_f64 != p_f64:
        v = 0
    elif p_f64 >= 9.223372036854775807e18:
        v = (1 << 63) - 1
    elif p_f64 <= -9.223372036854775808e18:
        v = -(1 << 63)
    else:
        v = int(p_f64)
    return (v * 1000000000) & ((1 << 64) - 1)


def main():
    kats = {
        "source": "al8n/ruserf @ v2 (read-only reference); values transcribed from its unit tests",
        "coordinate": {
            "opts_default": {
                "ref": "core/src/coordinate.rs:200-213",
                "dimensionality": 8, "vivaldi_error_max": 1.5, "vivaldi_ce": 0.25,
                "vivaldi_cc": 0.25, "adjustment_window_size": 20, "height_min": 10.0e-6,
                "latency_filter_size": 3, "gravity_rho": 150.0,
            },
            "zero_threshold": {"ref": "core/src/coordinate.rs:18,829-833", "value": 1.0e-6},
            "client_update": {
                "ref": "core/src/coordinate.rs:886-911",
                "dim": 3, "other_portion": [0.0, 0.0, 0.001],
                "rtt_ns": int(2.0 * 0.001 * 1.0e9),
                "expect": "portion[2] < 0; then set_coordinate(portion[2]=99) reads back 99",
            },
            "client_invalid_in_ping_values": {
                "ref": "core/src/coordinate.rs:913-938",
                "dim": 3, "other_portion": [0.0, 0.0, 0.001],
                "pings_f64": [9223372036854775807.0, -35.0, 11.0],
                "rtt_ns": [i64_wrapping_mul_as_u64(p) for p in [9223372036854775807.0, -35.0, 11.0]],
                "expect_error": "InvalidRTT", "expect": "distance_to(other) unchanged",
            },
            "client_distance_to": {
                "ref": "core/src/coordinate.rs:940-954",
                "dim": 3, "height_min": 0.0, "other_portion": [0.0, 0.0, 12.345],
                "expect_ns": int(12.345 * 1.0e9),
            },
            "client_latency_filter": {
                "ref": "core/src/coordinate.rs:956-1033",
                "filter_size": 3,
                "steps": [
                    ["alice", 0.201, 0.201], ["alice", 0.200, 0.201], ["alice", 0.207, 0.201],
                    ["alice", 1.9, 0.207], ["alice", 0.203, 0.207], ["alice", 0.199, 0.203],
                    ["alice", 0.211, 0.203], ["bob", 0.310, 0.310],
                    ["forget", "alice", None], ["alice", 0.888, 0.888],
                ],
            },
            "client_nan_defense": {
                "ref": "core/src/coordinate.rs:1035-1067",
                "dim": 3, "rtt_ns": 250 * 1000 * 1000,
                "expect": ["update(other with NaN) -> InvalidCoordinate",
                           "set_coordinate(dim 6) -> DimensionalityMismatch",
                           "poisoned self + update -> Ok, valid, resets == 1"],
            },
            "coordinate_apply_force": {
                "ref": "core/src/coordinate.rs:1108-1158",
                "dim": 3,
                "note": "`above` is built with height_min 0 (line 1119), so its height stays 0 in the last two cases",
                "cases": [
                    {"height_min": 0.0, "self": [0.0, 0.0, 0.0], "self_height": 0.0,
                     "force": 5.3, "other": [0.0, 0.0, 2.9], "other_height": 0.0,
                     "expect_portion": [0.0, 0.0, -5.3]},
                    {"height_min": 0.0, "self": [0.0, 0.0, -5.3], "self_height": 0.0,
                     "force": 2.0, "other": [3.4, 0.0, -5.3], "other_height": 0.0,
                     "expect_portion": [-2.0, 0.0, -5.3]},
                    {"height_min": 10.0e-6, "self": [0.0, 0.0, 0.0], "self_height": 10.0e-6,
                     "force": 5.3, "other": [0.0, 0.0, 2.9], "other_height": 0.0,
                     "expect_portion": [0.0, 0.0, -5.3],
                     "expect_height": 10.0e-6 + 5.3 * 10.0e-6 / 2.9},
                    {"height_min": 10.0e-6, "self": [0.0, 0.0, 0.0], "self_height": 10.0e-6,
                     "force": -5.3, "other": [0.0, 0.0, 2.9], "other_height": 0.0,
                     "expect_portion": [0.0, 0.0, 5.3], "expect_height": 10.0e-6},
                ],
                "random_case": {"height_min": 0.0, "force": 1.0,
                                "expect_distance_secs": 1.0},
                "panic_case": "dimension mismatch -> 'coordinate dimensionality does not match'",
            },
            "coordinate_add": {"ref": "core/src/coordinate.rs:1160-1171",
                               "a": [1.0, -3.0, 3.0], "b": [-4.0, 5.0, 6.0],
                               "expect": [-3.0, 2.0, 9.0]},
            "coordinate_diff": {"ref": "core/src/coordinate.rs:1173-1181",
                                "a": [1.0, -3.0, 3.0], "b": [-4.0, 5.0, 6.0],
                                "expect": [5.0, -8.0, -3.0]},
            "coordinate_magnitude": {"ref": "core/src/coordinate.rs:1199-1206",
                                     "v": [1.0, -2.0, 3.0], "expect": 3.7416573867739413},
            "coordinate_unit_vector_at": {
                "ref": "core/src/coordinate.rs:1208-1227",
                "a": [1.0, 2.0, 3.0], "b": [0.5, 0.6, 0.7],
                "expect": [0.18257418583505536, 0.511207720338155, 0.8398412548412546],
            },
            "codec_layout": {"ref": "core/src/coordinate.rs:663-745",
                             "layout": "u32be len | f64be error | f64be adjustment | f64be height | f64be portion[]",
                             "encoded_len": "4 + 8*dim + 24"},
        },
        "clock": {
            "ref": "types/src/clock.rs:192-208",
            "ops": [["time", 0], ["increment", 1], ["time", 1], ["witness", 41, 42],
                    ["witness", 41, 42], ["witness", 30, 42]],
        },
        "merge": {
            "serf_reap_handler": {
                "ref": "core/src/serf/base/tests/serf/reap.rs:41-131 (Reaper::run, base.rs:580-601)",
                "tombstone_timeout_s": 6, "recent_intent_timeout_s": 7,
                # left_members entries with leave_time = now - age
                "left_ages_s": [0, 5, 10], "expect_left_remaining": 2,
                # recent_intents: (node, type, ltime, age)
                "intents": [["alice", "join", 1, 0], ["bob", "join", 2, 10], ["carol", "leave", 1, 0],
                            ["doug", "leave", 2, 10]],
                "expect_intents_kept": ["alice", "carol"]},
            "join_intent_buffer_early": {
                "ref": "core/src/serf/base/tests/serf/join.rs:8-35",
                "subject_known": False, "ltime": 10,
                "expect": [True, False], "buffered": ["join", 10]},
            "join_intent_old_message": {
                "ref": "core/src/serf/base/tests/serf/join.rs:38-87",
                "subject": ["alive", 12], "ltime": 10, "expect": False, "buffered": None},
            "join_intent_newer": {
                "ref": "core/src/serf/base/tests/serf/join.rs:90-138",
                "subject": ["alive", 12], "ltime": 14, "expect": True,
                "status_time": 14, "clock": 15},
            "join_intent_reset_leaving": {
                "ref": "core/src/serf/base/tests/serf/join.rs:141-191",
                "subject": ["leaving", 12], "ltime": 14, "expect": True,
                "status_time": 14, "status": "alive", "clock": 15},
            "join_pending_intent": {
                "ref": "core/src/serf/base/tests/serf/join.rs:273-310",
                "intents": [["join", 5]], "after_node_join": ["alive", 5]},
            "join_pending_intents": {
                "ref": "core/src/serf/base/tests/serf/join.rs:313-357",
                "intents": [["join", 5], ["leave", 6]], "after_node_join": ["leaving", 6]},
            "leave_intent_buffer_early": {
                "ref": "core/src/serf/base/tests/serf/leave.rs:4-32",
                "subject_known": False, "ltime": 10,
                "expect": [True, False], "buffered": ["leave", 10]},
            "leave_intent_old_message": {
                "ref": "core/src/serf/base/tests/serf/leave.rs:35-84",
                "subject": ["alive", 12], "ltime": 10, "expect": False, "buffered": None},
            "leave_intent_newer": {
                "ref": "core/src/serf/base/tests/serf/leave.rs:87-140",
                "subject": ["alive", 12], "ltime": 14, "expect": True,
                "status": "leaving", "clock": 15},
            "delegate_merge_remote_state": {
                "ref": "core/src/serf/base/tests/serf/delegate.rs:121-186 (driver: core/src/serf/delegate.rs:422-554)",
                "pp": {"ltime": 42, "status_ltimes": [["test", 20], ["foo", 15]],
                       "left_members": ["foo"], "event_ltime": 50,
                       "events": [[45, [["test", ""]]]], "query_ltime": 100},
                "expect": {"clock": 42, "intent_test": ["join", 20], "intent_foo": ["leave", 16],
                           "event_clock": 50, "event_slot_45_name": "test", "query_clock": 100}},
        },
        "dissemination": {
            "event_buffer_size": {"ref": "core/src/options.rs (event_buffer_size default)", "value": 512},
            "query_buffer_size": {"ref": "core/src/options.rs (query_buffer_size default)", "value": 512},
            "user_event_old_message": {
                "ref": "core/src/serf/base/tests/serf/event.rs:6-29",
                "witness": 512 + 1000, "ltime": 1, "expect": False},
            "user_event_same_clock": {
                "ref": "core/src/serf/base/tests/serf/event.rs:32-74",
                "events": [[1, "first", "test"], [1, "first", "newpayload"], [1, "second", "other"]],
                "expect": [True, True, True],
                "delivered": [["first", "test"], ["first", "newpayload"], ["second", "other"]]},
            "query_old_message": {
                "ref": "core/src/serf/base/tests/serf/event.rs:653-687",
                "witness": 512 + 1000, "ltime": 1, "id": 0, "expect": False},
            "query_same_clock": {
                "ref": "core/src/serf/base/tests/serf/event.rs:690-775",
                "queries": [[1, 1, "foo"], [1, 1, "foo"], [1, 2, "bar"], [1, 2, "bar"],
                            [1, 3, "baz"], [1, 3, "baz"]],
                "expect": [True, False, True, False, True, False],
                "delivered": ["foo", "bar", "baz"]},
            "user_event_coalesce_basic": {
                "ref": "core/src/coalesce/user.rs:125-200",
                "events": [["foo", 1, ""], ["foo", 2, ""], ["bar", 2, "test1"], ["bar", 2, "test2"]],
                "expect_flushed": [["foo", 2, ""], ["bar", 2, "test1"], ["bar", 2, "test2"]]},
            # origination size limits: Serf::user_event (core/src/serf/api.rs:255-287) and
            # query_in (core/src/serf/base.rs:916-921) against Options' defaults
            # (core/src/options.rs:519, 526; test_config leaves both at the default,
            # core/src/serf/base/tests.rs:27-41)
            "max_user_event_size": {"ref": "core/src/options.rs:526", "value": 512},
            "query_size_limit": {"ref": "core/src/options.rs:519", "value": 1024},
            "user_event_size_limit_const": {"ref": "core/src/serf.rs:42", "value": 9 * 1024},
            "serf_event_user_size_limit": {
                "ref": "core/src/serf/base/tests/serf/event.rs:506-525",
                "name": "this is too large an event", "payload_len": "max_user_event_size",
                "expect_error_contains": "user event exceeds"},
            "serf_query_size_limit": {
                "ref": "core/src/serf/base/tests/serf/event.rs:1070-1085",
                "name": "this is too large a query", "payload_len": "query_size_limit",
                "query_size_limit_factor": 1, "expect_error_contains": "query exceeds limit of"},
            "serf_query_size_limit_increased": {
                "ref": "core/src/serf/base/tests/serf/event.rs:1087-1100",
                "name": "this is too large a query", "payload_len": "query_size_limit",
                "query_size_limit_factor": 2, "expect_ok": True},
        },
    }
    out = os.path.join(HERE, "reference_kats.json")
    with open(out, "w") as f:
        json.dump(kats, f, indent=1, sort_keys=True)
        f.write("\n")
    print("wrote", out)


if __name__ == "__main__":
    main()
